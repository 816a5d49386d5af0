"""Time each fused-MLP kernel in isolation at the cfg#2 fine-net size (HIP events)."""
import ctypes, sys, torch
sys.path[:0] = [".", "robust-nerf_amd"]
from noisy_src import _hip
_hip.load(require_all=False)  # NR_HIP_LIB may name an older library (A/B runs)
from noisy_src.config import ModelConfig
from noisy_src.model import NeRF
MACS = 593408
def bench(prec, M, reps=int(__import__("os").environ.get("MB_REPS", "20"))):
    torch.manual_seed(0)
    net = NeRF(ModelConfig(precision=prec)).cuda()
    net._ensure_flat(); packed = net._packed_for_forward(); flat = net._flat
    cfg = ctypes.byref(net._nr_cfg); L = _hip.load(); st = _hip.stream_ptr()
    x = torch.rand(M, 3, device="cuda") * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(M, 3, device="cuda"), dim=-1)
    rgb = torch.empty(M, 3, device="cuda"); sig = torch.empty(M, 1, device="cuda")
    saved = torch.empty(L.nr_mlp_saved_bytes(cfg, M), dtype=torch.uint8, device="cuda")
    ws = torch.empty(L.nr_mlp_workspace_bytes(cfg, M), dtype=torch.uint8, device="cuda")
    grgb = torch.randn(M, 3, device="cuda"); gs = torch.randn(M, 1, device="cuda")
    # MB_ACTIVE=f: zero the incoming gradient of all but a fraction f of the 32-sample tiles
    # (the trained-state regime: the backward then runs on the active tiles only)
    # MB_PATTERN=rays: whole rays of MB_TPR tiles (default 6: 192 samples) are active in
    # their tiles 1..MB_TPR-1 with probability f / ((MB_TPR-1)/MB_TPR) (a trained field's
    # shape: rays that miss have no active tile, rays that hit one run of them)
    f = float(__import__("os").environ.get("MB_ACTIVE", "1"))
    if f < 1:
        T = (M + 31) // 32
        if __import__("os").environ.get("MB_PATTERN") == "rays":
            tpr = int(__import__("os").environ.get("MB_TPR", "6"))
            hit = torch.rand((T + tpr - 1) // tpr, device="cuda") < f * tpr / (tpr - 1)
            run = torch.ones(tpr, dtype=torch.bool, device="cuda"); run[0] = False
            tk = (hit[:, None] & run[None, :]).reshape(-1)[:T]
        else:
            tk = torch.rand(T, device="cuda") < f
        keep = tk.repeat_interleave(32)[:M]
        grgb *= keep[:, None]; gs *= keep[:, None]
    gflat = torch.empty_like(flat)
    P = _hip.ptr
    fns = {
        "fwd_infer": lambda: _hip.call("nr_mlp_forward", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig), None, st),
        "fwd_train": lambda: _hip.call("nr_mlp_forward", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig), P(saved), st),
        "bwd_dx": lambda: _hip.call("nr_mlp_backward_dx", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig), P(saved), P(grgb), P(gs), None, None, P(ws), st),
        "bwd_dw": lambda: _hip.call("nr_mlp_backward_dw", cfg, M, P(saved), P(ws), st),
        "bwd_reduce": lambda: _hip.call("nr_mlp_backward_reduce", cfg, M, P(ws), P(gflat), st),
    }
    out = {}
    names = __import__("os").environ.get("MB_KERNELS", "fwd_infer,fwd_train,bwd_dx,bwd_dw,bwd_reduce")
    for name in names.split(","):
        fn = fns[name]
        fn(); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps): fn()
        e.record(); torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        tf = 2 * MACS * M / (ms * 1e-3) / 1e12
        out[name] = ms
        print(f"{prec} M={M} {name:10s} {ms:8.3f} ms  {tf:7.1f} TF/s-equiv")
    return out
# MB_M: comma-separated sample counts (default the cfg #2 fine net)
for prec in sys.argv[1:] or ["bf16"]:
    for M in [int(v) for v in __import__("os").environ.get("MB_M", "786432").split(",")]:
        bench(prec, M)
