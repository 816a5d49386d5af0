"""A/B: the fine and coarse MLP backward chains (dX -> dW -> reduce) run one after the
other on one stream, or concurrently on two streams (they are independent: the
coarse net's backward does not depend on the fine net's).  cfg #2 sizes, bf16."""
import ctypes, os, sys, torch
sys.path[:0] = [".", "robust-nerf_amd"]
from noisy_src import _hip
from noisy_src.config import ModelConfig
from noisy_src.model import NeRF

REPS = int(os.environ.get("MB_REPS", "10"))
L = _hip.load()
P = _hip.ptr


def setup(M, seed):
    torch.manual_seed(seed)
    net = NeRF(ModelConfig(precision="bf16")).cuda()
    net._ensure_flat(); packed = net._packed_for_forward(); flat = net._flat
    cfg = ctypes.byref(net._nr_cfg)
    x = torch.rand(M, 3, device="cuda") * 3 - 1.5
    d = torch.nn.functional.normalize(torch.randn(M, 3, device="cuda"), dim=-1)
    rgb = torch.empty(M, 3, device="cuda"); sig = torch.empty(M, 1, device="cuda")
    saved = torch.empty(L.nr_mlp_saved_bytes(cfg, M), dtype=torch.uint8, device="cuda")
    ws = torch.empty(L.nr_mlp_workspace_bytes(cfg, M), dtype=torch.uint8, device="cuda")
    grgb = torch.randn(M, 3, device="cuda") * 1e-4; gs = torch.randn(M, 1, device="cuda") * 1e-4
    gflat = torch.empty_like(flat)
    st0 = _hip.stream_ptr()
    _hip.call("nr_mlp_forward", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig), P(saved), st0)

    def dx(st):
        _hip.call("nr_mlp_backward_dx", cfg, P(packed), P(flat), P(x), P(d), M, P(rgb), P(sig), P(saved), P(grgb),
                  P(gs), None, None, P(ws), st)

    def dw(st):
        _hip.call("nr_mlp_backward_dw", cfg, M, P(saved), P(ws), st)
        _hip.call("nr_mlp_backward_reduce", cfg, M, P(ws), P(gflat), st)
    keep = (net, packed, flat, x, d, rgb, sig, saved, ws, grgb, gs, gflat)
    return dx, dw, keep


fine_dx, fine_dw, kf = setup(786432, 0)
coarse_dx, coarse_dw, kc = setup(262144, 1)
s_main = torch.cuda.current_stream()
s_side = torch.cuda.Stream()
pm, ps = s_main.cuda_stream, s_side.cuda_stream


def sequential():
    fine_dx(pm); fine_dw(pm); coarse_dx(pm); coarse_dw(pm)


def two_streams():
    # side stream: the coarse chain, started together with the fine chain
    ev = torch.cuda.Event(); ev.record(s_main); s_side.wait_event(ev)
    fine_dx(pm); coarse_dx(ps); fine_dw(pm); coarse_dw(ps)
    ev2 = torch.cuda.Event(); ev2.record(s_side); s_main.wait_event(ev2)


def coarse_after_fine_dx():
    # coarse dX waits for the fine dX, then runs beside the fine dW
    fine_dx(pm)
    ev = torch.cuda.Event(); ev.record(s_main); s_side.wait_event(ev)
    coarse_dx(ps); fine_dw(pm); coarse_dw(ps)
    ev2 = torch.cuda.Event(); ev2.record(s_side); s_main.wait_event(ev2)


def fine_dw_last():
    # fine dX, then coarse dX + coarse dW on the side beside the fine dW
    fine_dx(pm); coarse_dx(pm)
    ev = torch.cuda.Event(); ev.record(s_main); s_side.wait_event(ev)
    coarse_dw(ps); fine_dw(pm)
    ev2 = torch.cuda.Event(); ev2.record(s_side); s_main.wait_event(ev2)


for name, fn in (("sequential", sequential), ("two_streams", two_streams),
                 ("coarse_after_fine_dx", coarse_after_fine_dx), ("fine_dw_last", fine_dw_last),
                 ("sequential", sequential)):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record(); torch.cuda.synchronize()
    print(f"overlap {name:22s} {s.elapsed_time(e) / REPS:8.3f} ms per backward (fine+coarse)", flush=True)
