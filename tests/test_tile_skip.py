"""GPU: the backward skips 32-sample tiles whose incoming gradient is exactly zero
(csrc/mlp.hip tile_flags_kernel / select_tile).

A sample with sigma == 0 (alpha = w = 0 and ReLU'(0) = 0, reference rendering.py:83) or
with its transmittance underflowed to 0 (cumprod of 1 - alpha + 1e-10, rendering.py:87-96)
receives exactly zero g_rgb / g_sigma, so every layer's dz for it is zero and a tile of
such samples adds only exact zeros to dW.  The skipping form is checked against the
dense one (NrMlpConfig.dense_backward = 1, which runs every tile as the reference's full
backward does):

* every tile active: bit-identical (same work list, same chunk split);
* >= 50 % of the tiles inactive: input gradients bit-identical (per-sample work), the
  parameter gradient equal up to the dW chunk split's summation order;
* no tile active: exactly zero gradients;
* the same on a trained state through the whole render + backward (the zeros come from the
  compositing itself there), and the count the kernels ran on equals the tiles with a
  nonzero incoming gradient."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net(precision, seed=0, **kw):
    from noisy_src.config import ModelConfig
    from noisy_src.model import NeRF
    torch.manual_seed(seed)
    return NeRF(ModelConfig(precision=precision, **kw)).to(DEV)


def _inputs(M, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(M, 3, generator=g) * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
    gr = torch.randn(M, 3, generator=g) * 1e-3
    gs = torch.randn(M, 1, generator=g) * 1e-3
    return [t.to(DEV) for t in (x, d, gr, gs)]


def _backward(net, x, d, gr, gs, dense, inputs=False):
    net._nr_cfg.dense_backward = int(dense)
    net._tile_counts = []
    xx = x.clone().requires_grad_(inputs)
    dd = d.clone().requires_grad_(inputs)
    rgb, sig = net(xx, dd)
    net.zero_grad(set_to_none=True)
    torch.autograd.backward([rgb, sig], [gr, gs])
    g = torch.cat([p.grad.reshape(-1) for p in net.parameters()]).clone()
    (M, cnt), = net._tile_counts
    net._tile_counts = None
    net._nr_cfg.dense_backward = 0
    return g, (xx.grad, dd.grad) if inputs else None, int(cnt.item())


def _expected_active(gr, gs):
    M = gr.shape[0]
    nz = (gr != 0).any(-1) | (gs.reshape(-1) != 0)
    pad = (-M) % 32
    return int(torch.nn.functional.pad(nz, (0, pad)).reshape(-1, 32).any(-1).sum())


def _zero_tiles(gr, gs, frac, seed=5):
    """Zero the incoming gradient of a random `frac` of the tiles, and of a few single
    samples inside the kept ones."""
    M = gr.shape[0]
    T = (M + 31) // 32
    g = torch.Generator().manual_seed(seed)
    dead = (torch.rand(T, generator=g) < frac).repeat_interleave(32)[:M].to(DEV)
    lone = (torch.rand(M, generator=g) < 0.3).to(DEV)
    keep = ~(dead | lone)
    return gr * keep[:, None], gs * keep[:, None]


@pytest.mark.parametrize("precision", ["bf16", "fp16", "fp32"])
def test_all_tiles_active_is_bit_identical(precision):
    M = 60_003 if precision != "fp32" else 20_003  # a partial last tile
    net = _net(precision)
    x, d, gr, gs = _inputs(M)
    gd, ind, cd = _backward(net, x, d, gr, gs, dense=True, inputs=True)
    gk, ink, ck = _backward(net, x, d, gr, gs, dense=False, inputs=True)
    assert cd == ck == (M + 31) // 32
    assert torch.equal(gd, gk)
    assert torch.equal(ind[0], ink[0]) and torch.equal(ind[1], ink[1])


@pytest.mark.parametrize("precision,M", [("bf16", 98_304), ("fp16", 98_304), ("fp32", 24_576),
                                         # ragged: a partial last segment / a partial last tile
                                         ("bf16", 70_001), ("bf16", 8_225), ("fp32", 9_001)])
def test_half_the_tiles_inactive(precision, M):
    net = _net(precision, seed=2)
    x, d, gr, gs = _inputs(M, seed=3)
    gr, gs = _zero_tiles(gr, gs, 0.6)
    want = _expected_active(gr, gs)
    assert want <= 0.5 * ((M + 31) // 32)
    gd, ind, cd = _backward(net, x, d, gr, gs, dense=True, inputs=True)
    gk, ink, ck = _backward(net, x, d, gr, gs, dense=False, inputs=True)
    assert cd == (M + 31) // 32 and ck == want
    # per-sample work: identical; inactive samples' input gradients exactly zero
    assert torch.equal(ind[0], ink[0]) and torch.equal(ind[1], ink[1])
    # dW: the same products, summed in another chunk grouping (fp32 accumulation)
    err = (gd - gk).abs().max().item()
    assert err <= 1e-4 * gd.abs().max().item(), err
    rel = ((gd - gk).norm() / gd.norm()).item()
    assert rel < 1e-5, rel


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_no_tile_active_gives_zero(precision):
    M = 4_096
    net = _net(precision)
    x, d, gr, gs = _inputs(M)
    gr, gs = torch.zeros_like(gr), torch.zeros_like(gs)
    gk, ink, ck = _backward(net, x, d, gr, gs, dense=False, inputs=True)
    gd, ind, _ = _backward(net, x, d, gr, gs, dense=True, inputs=True)
    assert ck == 0
    assert not gk.any() and not gd.any()
    assert not ink[0].any() and not ink[1].any()


@pytest.mark.parametrize("M", [33, 1_000, 40_000])
def test_single_active_tile(M):
    """One active tile (the last, possibly partial one) among inactive ones: the dX
    workgroup of its segment runs it with seven idle waves; gradients equal the dense ones
    (one tile: the same products in the same order)."""
    net = _net("bf16", seed=4)
    x, d, gr, gs = _inputs(M, seed=6)
    T = (M + 31) // 32
    keep = torch.zeros(M, dtype=torch.bool, device=DEV)
    keep[(T - 1) * 32:] = True
    gr, gs = gr * keep[:, None], gs * keep[:, None]
    gd, ind, cd = _backward(net, x, d, gr, gs, dense=True, inputs=True)
    gk, ink, ck = _backward(net, x, d, gr, gs, dense=False, inputs=True)
    assert ck == 1 and cd == T
    assert torch.equal(ind[0], ink[0]) and torch.equal(ind[1], ink[1])
    err = (gd - gk).abs().max().item()
    assert err <= 1e-5 * gd.abs().max().item(), err


def test_launch_past_the_dense_check():
    """Past kDenseCheckSegs (1,024) segments of 256 tiles (M > 8,388,608 samples) the dX
    workgroups skip the all-active check, which would read every block count in every
    workgroup, and always take the segment-minor form (leaders alone read the counts
    before their segment).  Both the dense form (every tile flagged) and the skipping one
    run that way: same input gradients bit for bit, dW to summation order, right count."""
    M = 1_025 * 8_192 + 77  # 1,026 segments, a ragged last one
    T = (M + 31) // 32
    net = _net("bf16", seed=8)
    x, d, gr, gs = _inputs(M, seed=9)
    gr, gs = _zero_tiles(gr, gs, 0.5, seed=10)
    want = _expected_active(gr, gs)
    gd, ind, cd = _backward(net, x, d, gr, gs, dense=True, inputs=True)
    gk, ink, ck = _backward(net, x, d, gr, gs, dense=False, inputs=True)
    assert cd == T and ck == want
    assert torch.equal(ind[0], ink[0]) and torch.equal(ind[1], ink[1])
    rel = ((gd - gk).norm() / gd.norm()).item()
    assert rel < 1e-5, rel


def test_nan_gradient_keeps_its_tile():
    """A NaN incoming gradient is not zero: its tile runs (and the NaN reaches dW)."""
    M = 3_200
    net = _net("bf16")
    x, d, gr, gs = _inputs(M)
    gr, gs = torch.zeros_like(gr), torch.zeros_like(gs)
    gs[1_000] = float("nan")
    gk, _, ck = _backward(net, x, d, gr, gs, dense=False)
    assert ck == 1 and torch.isnan(gk).any()


def test_trained_state_backward_matches_dense():
    """The cfg #2 render + losses + backward on a trained sphere-scene state (bench.py's
    trained leg, fewer iterations): most tiles are inactive because of the compositing
    itself; the skipping backward's gradients equal the dense ones up to the dW chunk
    split's summation order, and the kernels ran on exactly the tiles with a nonzero
    incoming gradient."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from noisy_src import ops
    from noisy_src.rendering import render_rays
    tr, (o, d, gt), n_train = bench.train_sphere_state("bf16", torch.device(DEV), iters=600)
    g = torch.Generator(device=DEV).manual_seed(9)
    idx = torch.randint(0, n_train, (4096,), device=DEV, generator=g)
    rc = tr.render_config
    t_rand = torch.rand(4096, rc.num_samples, device=DEV, generator=g)
    u = torch.rand(4096, rc.num_samples_fine, device=DEV, generator=g)
    nets = (tr.model_coarse, tr.model_fine)
    probe = {}

    def one(dense):
        for net in nets:
            net._nr_cfg.dense_backward = int(dense)
            net._tile_counts = []
            net.zero_grad(set_to_none=True)
        out = render_rays(*nets, o[idx], d[idx], rc, is_train=True, t_rand=t_rand, u=u)
        loss = ops.mse_loss(out["rgb_coarse"], gt[idx]) + ops.mse_loss(out["rgb_fine"], gt[idx])
        loss.backward()
        counts = {M: int(c.item()) for net in nets for M, c in net._tile_counts}
        for net in nets:
            net._tile_counts = None
            net._nr_cfg.dense_backward = 0
        return float(loss.detach()), [torch.cat([p.grad.reshape(-1) for p in net.parameters()]).clone() for net in nets], counts

    # the incoming gradients themselves, for the expected counts
    from noisy_src import model as model_mod
    orig = model_mod._MLPFunction.backward

    def spy(ctx, g_rgb, g_sigma):
        probe[g_rgb.shape[0]] = _expected_active(g_rgb, g_sigma)
        return orig(ctx, g_rgb, g_sigma)

    model_mod._MLPFunction.backward = staticmethod(spy)
    try:
        ld, gd, cd = one(True)
        lk, gk, ck = one(False)
    finally:
        model_mod._MLPFunction.backward = staticmethod(orig)
    assert ld == lk
    assert ck == probe, (ck, probe)
    assert all(cd[M] == (M + 31) // 32 for M in cd)
    assert max(ck[M] / ((M + 31) // 32) for M in ck) <= 0.6, ck
    for a, b in zip(gd, gk):
        assert ((a - b).norm() / a.norm()).item() < 1e-5
        assert (a - b).abs().max().item() <= 1e-4 * a.abs().max().item()
