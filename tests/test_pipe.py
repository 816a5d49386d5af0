"""The fused layer-pipelined backward (nr_mlp_backward_dxdw, csrc/mlp_pipe.inc) against
the split backward (nr_mlp_backward_dx then nr_mlp_backward_dw) through the C ABI.

Both run the same MFMA products in the same order per dW chunk, so the reduced flat
gradients (and, for pose optimisation, g_x / g_d) must be BIT-identical, at sizes from
one tile to the cfg #2 fine net (M = 786,432), for bf16 and fp16 and the model
variants the pipeline covers.  The split path itself is checked against the oracle by
test_parity_mlp.py / test_parity_fullsize.py.  Every pipelined call must also leave its
status word 0 (no bounded wait timed out)."""

import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _net(precision, skips=(4,), use_view_dirs=True, layers=8, seed=0, **extra):
    from noisy_src.config import ModelConfig
    from noisy_src.model import NeRF
    cfg = ModelConfig(precision=precision, skips=skips, use_view_dirs=use_view_dirs, num_hidden_layers=layers,
                      **extra)
    torch.manual_seed(seed)
    return NeRF(cfg).to(DEV)


def _run(net, M, seed=1, want_in=False):
    """(gflat split, gflat fused, g_x/g_d pairs, status word) for M samples."""
    from noisy_src import _hip
    from noisy_src._hip import call, ptr
    lib = _hip.load()
    cfg = ctypes.byref(net._nr_cfg)
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = (torch.rand(M, 3, device=DEV, generator=g) * 3 - 1.5).contiguous()
    d = torch.nn.functional.normalize(torch.randn(M, 3, device=DEV, generator=g), dim=-1).contiguous()
    use_d = net.config.use_view_dirs
    flat = net.flat_params()
    packed = net._packed_for_forward()
    rgb = torch.empty(M, 3, device=DEV)
    sig = torch.empty(M, 1, device=DEV)
    saved = torch.empty(int(lib.nr_mlp_saved_bytes(cfg, M)), device=DEV, dtype=torch.uint8)
    st = _hip.stream_ptr()
    call("nr_mlp_forward", cfg, ptr(packed), ptr(flat), ptr(x), ptr(d) if use_d else None, M, ptr(rgb), ptr(sig),
         ptr(saved), st)
    g_rgb = torch.randn(M, 3, device=DEV, generator=g) * 1e-3
    g_sig = torch.randn(M, 1, device=DEV, generator=g) * 1e-3
    out = []
    for fused in (False, True):
        ws = torch.full((int(lib.nr_mlp_workspace_bytes(cfg, M)),), 0x7F, device=DEV, dtype=torch.uint8)  # poisoned
        gflat = torch.empty(net._param_count, device=DEV)
        gx = torch.empty(M, 3, device=DEV) if want_in else None
        gd = torch.empty(M, 3, device=DEV) if (want_in and use_d) else None
        args = (cfg, ptr(packed), ptr(flat), ptr(x), ptr(d) if use_d else None, M, ptr(rgb), ptr(sig), ptr(saved),
                ptr(g_rgb), ptr(g_sig), ptr(gx), ptr(gd), ptr(ws), st)
        if fused:
            call("nr_mlp_backward_dxdw", *args)
        else:
            call("nr_mlp_backward_dx", *args)
            call("nr_mlp_backward_dw", cfg, M, ptr(saved), ptr(ws), st)
        call("nr_mlp_backward_reduce", cfg, M, ptr(ws), ptr(gflat), st)
        torch.cuda.synchronize()
        status = None
        if fused:
            off = int(lib.nr_mlp_pipe_status_offset(cfg, M))
            status = int(ws[off:off + 4].view(torch.int32).item()) if off >= 0 else None
        out.append((gflat, gx, gd, status))
    return out


def _check(net, M, want_in=False, expect_pipe=True):
    from noisy_src import _hip
    cfg = ctypes.byref(net._nr_cfg)
    assert int(_hip.load().nr_mlp_backward_pipelined(cfg, M)) == int(expect_pipe)
    (g0, x0, d0, _), (g1, x1, d1, status) = _run(net, M, want_in=want_in)
    if expect_pipe:
        assert status == 0, f"pipelined backward timed out (status {status})"
    assert torch.isfinite(g0).all() and g0.abs().max() > 0
    nbad = int((g0 != g1).sum())
    assert nbad == 0, f"{nbad} of {g0.numel()} gradient entries differ, max {float((g0 - g1).abs().max()):.3e}"
    if want_in:
        assert torch.equal(x0, x1)
        if d0 is not None:
            assert torch.equal(d0, d1)


@pytest.mark.parametrize("M", [1, 100, 32 * 16 * 25 + 7, 65536, 262_144])
def test_fused_equals_split_bf16(M):
    _check(_net("bf16"), M)


def test_fused_equals_split_fine_cfg2():
    """cfg #2's fine net: M = 4096 x 192 (25 pipelines x 983 tiles; > 2^31 bytes of rings + slabs offsets)."""
    _check(_net("bf16"), 786_432)


def test_fused_equals_split_fp16():
    _check(_net("fp16"), 50_000)


@pytest.mark.parametrize("kw", [dict(use_view_dirs=False), dict(skips=()), dict(layers=1, skips=()),
                                dict(layers=4, skips=(1,)), dict(layers=6, skips=(4,))])
def test_fused_equals_split_models(kw):
    _check(_net("bf16", **kw), 20_000)


def test_fused_input_gradients_pose_mode():
    """g_x / g_d (pose optimisation) from the dz images the pipeline also writes."""
    _check(_net("bf16"), 30_000, want_in=True)


def test_outside_envelope_runs_split():
    """fp32, two-skip and one-block-x_enc models (pos_freqs 4: no pipelined kernel
    instance) are not pipelined: dxdw runs the split form (same result), and
    nr_mlp_backward_pipelined says so."""
    _check(_net("fp32"), 5000, expect_pipe=False)
    _check(_net("bf16", pos_freqs=4), 5000, expect_pipe=False)
    _check(_net("bf16", layers=7, skips=(2, 5)), 5000, expect_pipe=False)
