"""GPU parity: the fused HIP NeRF MLP (fp32 and bf16 MFMA paths) vs the oracle's
nn.Module MLP with identical weights.  fp32 bar: |rgb|,|sigma| within 1e-4 abs
(BASELINE.json north_star); bf16 bar: operand rounding only (relative 3e-2)."""
import pytest
import torch

from oracle import refimpl as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(precision, seed=0, skips=(4,), use_view_dirs=True):
    from noisy_src.config import ModelConfig
    from noisy_src.model import NeRF
    cfg = ModelConfig(precision=precision, skips=skips, use_view_dirs=use_view_dirs)
    torch.manual_seed(seed)
    oracle = ref.NeRF(cfg)
    torch.manual_seed(seed)
    net = NeRF(cfg)
    net.load_state_dict(oracle.state_dict())
    return oracle, net.to(DEV)


def _inputs(M, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(M, 3, generator=g) * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(M, 3, generator=g), dim=-1)
    return x, d


def test_same_init_and_state_dict_keys():
    from noisy_src.model import NeRF
    torch.manual_seed(42)
    a = ref.NeRF()
    torch.manual_seed(42)
    b = NeRF()
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa) == list(sb)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("M", [1000, 32, 1, 4096])
def test_fp32_forward(M):
    oracle, net = _pair("fp32")
    x, d = _inputs(M)
    with torch.no_grad():
        rgb, sig = net(x.to(DEV), d.to(DEV))
        wr, ws = oracle(x, d)
    assert rgb.shape == (M, 3) and sig.shape == (M, 1)
    assert (rgb.cpu() - wr).abs().max() < 1e-4
    assert (sig.cpu() - ws).abs().max() < 1e-4


def _kink_free(oracle, x, d, eps=2e-6):
    """Samples whose fp64 ReLU pre-activations all stay >= eps away from 0.  A unit within
    rounding of the kink may legitimately switch sides between two fp32 implementations
    (different summation order), which changes that sample's gradient by O(1)."""
    o64 = ref.NeRF(oracle.config).double()
    o64.load_state_dict({k: v.double() for k, v in oracle.state_dict().items()})
    mins = []
    hooks = [m.register_forward_hook(lambda m, i, out: mins.append(out.abs().min(dim=-1).values))
             for m in list(o64.pts_linears) + [o64.dir_linear, o64.sigma_linear]]
    with torch.no_grad():
        o64(x.double(), None if d is None else d.double())
    for h in hooks:
        h.remove()
    return torch.stack(mins, -1).min(-1).values >= eps


def _grads(oracle, net, x, d, seed=3, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    M = x.shape[0]
    keep = _kink_free(oracle, x, d).float()[:, None]
    gr = torch.randn(M, 3, generator=g) * keep
    gs = torch.randn(M, 1, generator=g) * keep
    o = oracle
    if dtype == torch.float64:
        o = ref.NeRF(oracle.config).double()
        o.load_state_dict({k: v.double() for k, v in oracle.state_dict().items()})
    xr, dr = x.clone().to(dtype).requires_grad_(True), d.clone().to(dtype).requires_grad_(True)
    wr, ws = o(xr, dr)
    ((wr * gr.to(dtype)).sum() + (ws * gs.to(dtype)).sum()).backward()
    xg, dg = x.clone().to(DEV).requires_grad_(True), d.clone().to(DEV).requires_grad_(True)
    rgb, sig = net(xg, dg)
    ((rgb * gr.to(DEV)).sum() + (sig * gs.to(DEV)).sum()).backward()
    return o, xr, dr, xg, dg, keep


def test_fp32_backward():
    """dL/dW, dL/dx, dL/dd vs the fp64 oracle on kink-free samples: the HIP fp32 path
    must be as close to fp64 as torch's own fp32 path is (~1e-6 relative)."""
    oracle, net = _pair("fp32")
    x, d = _inputs(777)
    o64, xr, dr, xg, dg, keep = _grads(oracle, net, x, d, dtype=torch.float64)
    assert keep.mean() > 0.7
    for (name, pr), pg in zip(o64.named_parameters(), net.parameters()):
        a, b = pg.grad.double().cpu(), pr.grad
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert rel < 2e-5, (name, rel)
    for a, b in ((xg.grad, xr.grad), (dg.grad, dr.grad)):
        rel = ((a.double().cpu() - b).norm() / b.norm()).item()
        assert rel < 2e-5, rel


def test_bf16_forward_backward():
    """bf16 MFMA path vs the oracle with bf16-rounded operands (oracle.bf16_operand_nerf):
    same operand precision, fp32 accumulation; only summation order differs."""
    oracle, net = _pair("bf16")
    emu = ref.bf16_operand_nerf(oracle)
    x, d = _inputs(1500)
    with torch.no_grad():
        rgb, sig = net(x.to(DEV), d.to(DEV))
        er, es = emu(x, d)
        wr, ws = oracle(x, d)
    assert (rgb.cpu() - er).abs().max() < 1e-4
    assert (sig.cpu() - es).abs().max() < 1e-4
    assert (rgb.cpu() - wr).abs().max() < 3e-3  # vs fp32: bf16 operand rounding
    keep = _kink_free(oracle, x, d, eps=1e-3).float()[:, None]  # bf16 moves pre-activations ~1e-3
    g = torch.Generator().manual_seed(3)
    gr = torch.randn(1500, 3, generator=g) * keep
    gs = torch.randn(1500, 1, generator=g) * keep
    er, es = emu(x, d)
    ((er * gr).sum() + (es * gs).sum()).backward()
    rgb, sig = net(x.to(DEV), d.to(DEV))
    ((rgb * gr.to(DEV)).sum() + (sig * gs.to(DEV)).sum()).backward()
    for (name, pe), pg in zip(emu.named_parameters(), net.parameters()):
        a, b = pg.grad.cpu(), pe.grad
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        # dz is stored in bf16 for the dW GEMM (the emulation keeps it fp32): <= ~1 bf16 ulp
        assert rel < 1e-2, (name, rel)


def test_fp16_forward_backward():
    """fp16 MFMA path (BASELINE cfg #5) vs the oracle with fp16-rounded operands.  The
    backward runs on dz scaled by 2^14 (undone exactly in the dW reduce); upstream
    gradients have the magnitude of a mean loss over 4096 rays."""
    oracle, net = _pair("fp16")
    emu = ref.fp16_operand_nerf(oracle)
    x, d = _inputs(1500)
    with torch.no_grad():
        rgb, sig = net(x.to(DEV), d.to(DEV))
        er, es = emu(x, d)
        wr, ws = oracle(x, d)
    assert (rgb.cpu() - er).abs().max() < 1e-4
    assert (sig.cpu() - es).abs().max() < 1e-4
    assert (rgb.cpu() - wr).abs().max() < 1e-3  # vs fp32: fp16 operand rounding
    keep = _kink_free(oracle, x, d, eps=1e-3).float()[:, None]
    g = torch.Generator().manual_seed(3)
    scale = 2.0 / (3 * 4096)
    gr = torch.randn(1500, 3, generator=g) * keep * scale
    gs = torch.randn(1500, 1, generator=g) * keep * scale
    er, es = emu(x, d)
    ((er * gr).sum() + (es * gs).sum()).backward()
    rgb, sig = net(x.to(DEV), d.to(DEV))
    ((rgb * gr.to(DEV)).sum() + (sig * gs.to(DEV)).sum()).backward()
    for (name, pe), pg in zip(emu.named_parameters(), net.parameters()):
        a, b = pg.grad.cpu(), pe.grad
        assert torch.isfinite(a).all(), name
        rel = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        # dz is stored in fp16 for the dW GEMM: <= ~1 fp16 ulp (2^-11)
        assert rel < 3e-3, (name, rel)


def test_no_view_dirs_and_other_skips():
    oracle, net = _pair("fp32", skips=(2,), use_view_dirs=False)
    x, _ = _inputs(300)
    with torch.no_grad():
        rgb, sig = net(x.to(DEV))
        wr, ws = oracle(x)
    assert (rgb.cpu() - wr).abs().max() < 1e-4
    assert (sig.cpu() - ws).abs().max() < 1e-4


def test_weights_update_repacks():
    """After an in-place parameter update the next forward uses the new weights."""
    oracle, net = _pair("fp32")
    x, d = _inputs(64)
    with torch.no_grad():
        net(x.to(DEV), d.to(DEV))
        for p, q in zip(net.parameters(), oracle.parameters()):
            p.mul_(0.5)
            q.mul_(0.5)
        rgb, sig = net(x.to(DEV), d.to(DEV))
        wr, ws = oracle(x, d)
    assert (rgb.cpu() - wr).abs().max() < 1e-4


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_16bit_input_gradients_vs_numerics_model(precision):
    """dL/dx and dL/dd (the pose-optimisation path's input gradients, WANT_X kernel
    variant) of the 16-bit MFMA path vs the numerics model (refimpl.MfmaEmulatedNeRF),
    on kink-free samples, at a mean-loss gradient scale.  The model computes x_enc with
    torch's sin; the kernels use the hardware sine (error ~1e-6), which moves a few
    x_enc values across a 16-bit rounding boundary, and those samples can then cross a
    ReLU kink downstream: per-sample agreement (p99) is tight, the norm over all samples
    carries those few outliers."""
    oracle, net = _pair(precision)
    emu = ref.mfma_emulated_nerf(oracle, precision)
    M = 20000
    x, d = _inputs(M, seed=5)
    # the model rounds like the kernels, so only summation-order flips (~1e-6) remain
    keep = _kink_free(oracle, x, d, eps=1e-5).float()[:, None]
    assert keep.mean() > 0.5
    g = torch.Generator().manual_seed(9)
    scale = 2.0 / (3 * 4096)
    gr = torch.randn(M, 3, generator=g) * keep * scale
    gs = torch.randn(M, 1, generator=g) * keep * scale
    xr, dr = x.clone().requires_grad_(True), d.clone().requires_grad_(True)
    er, es = emu(xr, dr)
    ((er * gr).sum() + (es * gs).sum()).backward()
    xg, dg = x.clone().to(DEV).requires_grad_(True), d.clone().to(DEV).requires_grad_(True)
    rgb, sig = net(xg, dg)
    ((rgb * gr.to(DEV)).sum() + (sig * gs.to(DEV)).sum()).backward()
    rx = ((xg.grad.cpu() - xr.grad).norm() / xr.grad.norm()).item()
    rd = ((dg.grad.cpu() - dr.grad).norm() / dr.grad.norm()).item()
    per = ((xg.grad.cpu() - xr.grad).norm(dim=-1) / xr.grad.norm(dim=-1).clamp_min(1e-30))
    print(f"{precision}: g_x rel {rx:.3e} (p99 per-sample {per.quantile(0.99).item():.3e}), g_d rel {rd:.3e}")
    assert per.quantile(0.99).item() < 2e-3, per.quantile(0.99).item()
    assert rx < 2e-2 and rd < 1e-2, (rx, rd)


_ODD_CONFIGS = {
    "no_view_dirs": dict(use_view_dirs=False),
    "pos6_dir2": dict(pos_freqs=6, dir_freqs=2),
    "depth7_skips2_5": dict(num_hidden_layers=7, skips=(2, 5)),
    "depth1": dict(num_hidden_layers=1, skips=()),
}


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
@pytest.mark.parametrize("name", sorted(_ODD_CONFIGS))
def test_16bit_non_default_configs_vs_numerics_model(precision, name):
    """the row-block-major 16-bit forward (odd-depth break path, skip chunk
    sizes, XB=1/DB=0 builds), the dX chain and the rearranged dW jobs for ModelConfigs
    other than the default 8x256/skip-4/view-dirs one, forward AND every parameter
    gradient vs the numerics model (refimpl.mfma_emulated_nerf) on kink-free samples
    at a mean-loss gradient scale."""
    from noisy_src.config import ModelConfig
    from noisy_src.model import NeRF
    cfg = ModelConfig(precision=precision, **_ODD_CONFIGS[name])
    torch.manual_seed(11)
    oracle = ref.NeRF(cfg)
    net = NeRF(cfg)
    net.load_state_dict(oracle.state_dict())
    net = net.to(DEV)
    emu = ref.mfma_emulated_nerf(oracle, precision)
    M = 3000
    x, d = _inputs(M, seed=13)
    dd = d if cfg.use_view_dirs else None
    with torch.no_grad():
        rgb, sig = net(x.to(DEV), None if dd is None else dd.to(DEV))
        er, es = emu(x, dd)
    assert (rgb.cpu() - er).abs().max() < 1e-4, name
    assert (sig.cpu() - es).abs().max() < 1e-3 * max(1.0, es.abs().max().item()), name
    # the model rounds like the kernels: only summation-order kink flips (~1e-6) remain
    keep = _kink_free(oracle, x, d if cfg.use_view_dirs else None, eps=1e-5).float()[:, None]
    assert keep.mean() > 0.5, keep.mean()
    g = torch.Generator().manual_seed(17)
    scale = 2.0 / (3 * 4096)
    gr = torch.randn(M, 3, generator=g) * keep * scale
    gs = torch.randn(M, 1, generator=g) * keep * scale
    er, es = emu(x, dd)
    ((er * gr).sum() + (es * gs).sum()).backward()
    rgb, sig = net(x.to(DEV), None if dd is None else dd.to(DEV))
    ((rgb * gr.to(DEV)).sum() + (sig * gs.to(DEV)).sum()).backward()
    # depth 1 has almost no ReLU kinks to flip: there the kernels equal the numerics
    # model to ~1e-5; deeper nets add kink flips that the hardware-sine vs torch-sine
    # encodings (a 16-bit rounding apart on a few values) trigger through the chain,
    # ~5e-3 uniformly over the layers (measured, tools/debug_cfg_grads.py)
    tol = 1e-3 if name == "depth1" else 1.5e-2
    rels = {}
    for (pname, pe), pg in zip(emu.base.named_parameters(), net.parameters()):
        a, b = pg.grad.cpu(), pe.grad
        assert torch.isfinite(a).all(), pname
        rels[pname] = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
    print(name, precision, "keep", round(keep.mean().item(), 3), "max grad rel", max(rels.values()))
    for pname, rel in rels.items():
        assert rel < tol, (name, pname, rel)
