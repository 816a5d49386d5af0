"""GPU: the training form of raw2outputs fused with the MSE loss (nr_composite_mse,
ops.composite_mse) against the three separate launches it replaces (nr_composite_fwd,
nr_mse_fwd_bwd, nr_composite_bwd through autograd) and against the oracle.  Reference:
rendering.py:20-116, train.py:89/98.  The gradients must be bit-identical to the
separate path; the loss value is the same mean summed in another order."""

import pytest
import torch

from oracle import refimpl as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(B, S, seed=0, zero_frac=0.3):
    g = torch.Generator().manual_seed(seed)
    rgb = torch.rand(B, S, 3, generator=g)
    sigma = torch.randn(B, S, 1, generator=g) * 3
    sigma[torch.rand(B, S, 1, generator=g) < zero_frac] = 0.0  # relu'(0) = 0 samples
    z = torch.sort(2 + 4 * torch.rand(B, S, generator=g), -1).values
    rd = torch.randn(B, 3, generator=g)
    tgt = torch.rand(B, 3, generator=g)
    return [t.to(DEV) for t in (rgb, sigma, z, rd, tgt)]


@pytest.mark.parametrize("S", [64, 192, 130, 600])
@pytest.mark.parametrize("with_rd", [False, True])
def test_fused_equals_separate(S, with_rd):
    from noisy_src import ops
    B = 700
    rgb, sigma, z, rd, tgt = _inputs(B, S, seed=S)
    grads = []
    losses = []
    for fused in (False, True):
        a = rgb.clone().requires_grad_(True)
        s = sigma.clone().requires_grad_(True)
        d = rd.clone().requires_grad_(with_rd)
        if fused:
            loss, rgb_map, *_ = ops.composite_mse(a, s, z, d, tgt, grad_scale=0.5)
        else:
            rgb_map = ops.composite(a, s, z, d)[0]
            loss = ops.mse_loss(rgb_map, tgt, 0.5)
        loss.backward(ops.unit_grad(torch.device(DEV)))
        grads.append([a.grad, s.grad] + ([d.grad] if with_rd else []))
        losses.append(loss.item())
    for x, y in zip(*grads):
        assert torch.equal(x, y)
    assert abs(losses[0] - losses[1]) <= 1e-6 * abs(losses[0])


def test_fused_matches_oracle_and_extra_output_grads():
    """Against the oracle's raw2outputs + MSE (fp32 torch); and a second use of rgb_map /
    the weights in the loss adds its own composite backward."""
    from noisy_src import ops
    B, S = 300, 96
    rgb, sigma, z, rd, tgt = _inputs(B, S, seed=7)
    a = rgb.clone().requires_grad_(True)
    s = sigma.clone().requires_grad_(True)
    loss, rgb_map, depth, acc, w = ops.composite_mse(a, s, z, rd, tgt)
    (loss + 0.1 * depth.sum() + 0.01 * w.square().sum()).backward()
    a2 = rgb.cpu().clone().requires_grad_(True)
    s2 = sigma.cpu().clone().requires_grad_(True)
    out = ref.raw2outputs(a2, s2, z.cpu(), rd.cpu())
    l2 = torch.mean((out["rgb_map"] - tgt.cpu()) ** 2)
    (l2 + 0.1 * out["depth_map"].sum() + 0.01 * out["weights"].square().sum()).backward()
    assert abs(loss.item() - l2.item()) < 1e-6
    assert (rgb_map.cpu() - out["rgb_map"]).abs().max() < 1e-5
    for x, y in ((a.grad, a2.grad), (s.grad, s2.grad)):
        assert (x.cpu() - y).abs().max() <= 1e-4 * y.abs().max() + 1e-7


@pytest.mark.parametrize("B", [1, 3, 700, 4096])
def test_in_launch_loss_sum(B):
    """With a ticket the launch's last workgroup sums the loss: the same gradients, the
    same loss up to summation order, and the ticket back at zero after every call."""
    from noisy_src import ops
    S = 64
    rgb, sigma, z, rd, tgt = _inputs(B, S, seed=B)
    ticket = torch.zeros(4, device=DEV, dtype=torch.int32)
    outs = []
    for tk in (None, ticket, ticket):
        a = rgb.clone().requires_grad_(True)
        s = sigma.clone().requires_grad_(True)
        loss, *_ = ops.composite_mse(a, s, z, rd, tgt, ticket=tk)
        loss.backward()
        outs.append((loss.item(), a.grad, s.grad))
        assert int(ticket[0]) == 0
    ref_loss = torch.mean((ops.composite(rgb, sigma, z, rd)[0] - tgt) ** 2).item()
    for lo, ga, gs in outs[1:]:
        assert torch.equal(ga, outs[0][1]) and torch.equal(gs, outs[0][2])
        assert abs(lo - outs[0][0]) <= 1e-6 * abs(outs[0][0])
        assert abs(lo - ref_loss) <= 1e-6 * abs(ref_loss)
    assert outs[1][0] == outs[2][0]  # deterministic
