"""A/B of one fused-MLP build against another on the GPU (kernel-variant tooling).

    NR_HIP_LIB=<lib> python tools/fwd_ab.py save OUT.pt     # outputs of that build
    python tools/fwd_ab.py compare A.pt B.pt                 # bitwise comparison

For bf16 and fp16 at two sizes (cfg #2's fine M and a ragged M), runs the training
forward, backward dX / dW / reduce and the inference forward on seeded inputs and
saves rgb, sigma (both forwards) and the flat parameter gradient, plus the kernel
times (HIP events).  The gradient covers every saved activation and mask the
backward reads, without depending on the padding bytes a build leaves untouched.
"""
import ctypes
import sys

import torch

sys.path[:0] = [".", "robust-nerf_amd"]
from noisy_src import _hip  # noqa: E402
from noisy_src.config import ModelConfig  # noqa: E402
from noisy_src.model import NeRF  # noqa: E402


def run(prec, M, reps=10):
    torch.manual_seed(0)
    net = NeRF(ModelConfig(precision=prec)).cuda()
    net._ensure_flat()
    packed = net._packed_for_forward()
    flat = net._flat
    cfg = ctypes.byref(net._nr_cfg)
    L = _hip.load()
    st = _hip.stream_ptr()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(M, 3, device="cuda", generator=g) * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(M, 3, device="cuda", generator=g), dim=-1)
    grgb = torch.randn(M, 3, device="cuda", generator=g) * 1e-3
    gs = torch.randn(M, 1, device="cuda", generator=g) * 1e-3
    rgb = torch.empty(M, 3, device="cuda")
    sig = torch.empty(M, 1, device="cuda")
    rgb_i = torch.empty(M, 3, device="cuda")
    sig_i = torch.empty(M, 1, device="cuda")
    saved = torch.zeros(L.nr_mlp_saved_bytes(cfg, M), dtype=torch.uint8, device="cuda")
    ws = torch.zeros(L.nr_mlp_workspace_bytes(cfg, M), dtype=torch.uint8, device="cuda")
    gflat = torch.empty_like(flat)
    P = _hip.ptr
    fns = {
        "fwd_train": lambda: _hip.call("nr_mlp_forward", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig),
                                       P(saved), st),
        "bwd_dx": lambda: _hip.call("nr_mlp_backward_dx", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig),
                                    P(saved), P(grgb), P(gs), None, None, P(ws), st),
        "bwd_dw": lambda: _hip.call("nr_mlp_backward_dw", cfg, M, P(saved), P(ws), st),
        "bwd_reduce": lambda: _hip.call("nr_mlp_backward_reduce", cfg, M, P(ws), P(gflat), st),
        "fwd_infer": lambda: _hip.call("nr_mlp_forward", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb_i),
                                       P(sig_i), None, st),
    }
    times = {}
    for name, fn in fns.items():
        fn()
    torch.cuda.synchronize()
    out = {"rgb": rgb.clone(), "sigma": sig.clone(), "rgb_infer": rgb_i.clone(), "sigma_infer": sig_i.clone(),
           "grad": gflat.clone()}
    for name, fn in fns.items():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        times[name] = s.elapsed_time(e) / reps
    out["times"] = times
    print(f"{prec:5s} M={M:7d} " + " ".join(f"{k}={v:.4f}ms" for k, v in times.items()), flush=True)
    return {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in out.items()}


def main():
    if sys.argv[1] == "save":
        res = {}
        for prec in ("bf16", "fp16"):
            for M in (786432, 1000):
                res[f"{prec}_{M}"] = run(prec, M)
        torch.save(res, sys.argv[2])
    else:
        A, B = torch.load(sys.argv[2]), torch.load(sys.argv[3])
        ok = True
        for key in A:
            for t in ("rgb", "sigma", "rgb_infer", "sigma_infer", "grad"):
                a, b = A[key][t], B[key][t]
                eq = torch.equal(a, b)
                ok &= eq
                diff = (a - b).abs().max().item()
                print(f"{key:14s} {t:12s} equal={eq} max|diff|={diff:.3e}")
            ta, tb = A[key]["times"], B[key]["times"]
            print("   " + " ".join(f"{k}: {ta[k]:.4f} -> {tb[k]:.4f}" for k in ta))
        print("ALL EQUAL" if ok else "MISMATCH")


if __name__ == "__main__":
    main()
