"""Repeatability of the fused and the split backward: the same inputs many times, each
path's gradients compared with its own first result and with the other path's
(diagnostic for intermittent mismatches)."""

import ctypes
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "robust-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_pipe import DEV, _net  # noqa: E402


def main(M=12807, reps=40):
    from noisy_src import _hip
    from noisy_src._hip import call, ptr
    net = _net("bf16")
    lib = _hip.load()
    cfg = ctypes.byref(net._nr_cfg)
    g = torch.Generator(device=DEV).manual_seed(1)
    x = (torch.rand(M, 3, device=DEV, generator=g) * 3 - 1.5).contiguous()
    d = torch.nn.functional.normalize(torch.randn(M, 3, device=DEV, generator=g), dim=-1).contiguous()
    flat = net.flat_params()
    packed = net._packed_for_forward()
    rgb = torch.empty(M, 3, device=DEV)
    sig = torch.empty(M, 1, device=DEV)
    saved = torch.empty(int(lib.nr_mlp_saved_bytes(cfg, M)), device=DEV, dtype=torch.uint8)
    st = _hip.stream_ptr()
    call("nr_mlp_forward", cfg, ptr(packed), ptr(flat), ptr(x), ptr(d), M, ptr(rgb), ptr(sig), ptr(saved), st)
    g_rgb = torch.randn(M, 3, device=DEV, generator=g) * 1e-3
    g_sig = torch.randn(M, 1, device=DEV, generator=g) * 1e-3
    ws = torch.empty(int(lib.nr_mlp_workspace_bytes(cfg, M)), device=DEV, dtype=torch.uint8)
    off = int(lib.nr_mlp_pipe_status_offset(cfg, M))
    names = [(n, p.numel()) for n, p in net.named_parameters()]

    def run(fused):
        ws.fill_(0x7F)
        gflat = torch.empty(net._param_count, device=DEV)
        args = (cfg, ptr(packed), ptr(flat), ptr(x), ptr(d), M, ptr(rgb), ptr(sig), ptr(saved), ptr(g_rgb),
                ptr(g_sig), None, None, ptr(ws), st)
        if fused:
            call("nr_mlp_backward_dxdw", *args)
        else:
            call("nr_mlp_backward_dx", *args)
            call("nr_mlp_backward_dw", cfg, M, ptr(saved), ptr(ws), st)
        call("nr_mlp_backward_reduce", cfg, M, ptr(ws), ptr(gflat), st)
        torch.cuda.synchronize()
        status = int(ws[off:off + 4].view(torch.int32).item()) if fused else 0
        return gflat, status

    def where(a, b):
        bad = a != b
        out, o = [], 0
        for n, c in names:
            k = int(bad[o:o + c].sum())
            if k:
                out.append(f"{n}:{k}")
            o += c
        return " ".join(out)

    s0, _ = run(False)
    f0, _ = run(True)
    print(f"M={M}: first split vs first fused: {int((s0 != f0).sum())} differ  {where(s0, f0)}")
    nf = ns = 0
    for r in range(reps):
        s, _ = run(False)
        f, status = run(True)
        bs, bf = int((s != s0).sum()), int((f != f0).sum())
        if bs or bf or status:
            print(f"rep {r}: split vs split0 {bs} [{where(s, s0)}]  fused vs fused0 {bf} [{where(f, f0)}]  "
                  f"status {status}")
        ns += bs > 0
        nf += bf > 0
    print(f"M={M}: {reps} reps, split unstable {ns}, fused unstable {nf}")


if __name__ == "__main__":
    for m in (sys.argv[1:] or ["12807", "65536"]):
        main(int(m))
