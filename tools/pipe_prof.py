"""Per-stage timing of the fused pipelined backward (diagnostic build only).

Run with NR_HIP_LIB pointing at a library built by
    tools/build_variant.sh pipeprof -DNR_PIPE_PROF
Every workgroup's wave 0 splits its tile loop into segments (csrc/mlp_pipe.inc
PipeProf); this prints, per stage kind, the mean cycles per tile of each segment, the
spin counts, and the start / end spread of the stages (100-MHz real time)."""

import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "robust-nerf_amd"))

from noisy_src import _hip  # noqa: E402
from noisy_src._hip import call, ptr  # noqa: E402
from noisy_src.config import ModelConfig  # noqa: E402
from noisy_src.model import NeRF  # noqa: E402

# segments of the v2 stage loops (csrc/mlp_pipe.inc, pf.seg(i)): trunk/feat 2 3 4 5 6 7,
# dir 2 10 3 4 5 7 8, x 2 3 4 6 7
SEG = {2: "top-wait", 3: "bar+sig", 4: "store+rdy", 5: "dX", 6: "poll+ld", 7: "dW|poll+ld", 8: "dW",
       9: "-", 10: "heads"}
KIND = {0: "dir", 1: "feat", 2: "trunk", 3: "x"}


def main(M=786_432, reps=3):
    dev = "cuda"
    lib = _hip.load()
    torch.manual_seed(0)
    net = NeRF(ModelConfig(precision="bf16")).to(dev)
    cfg = ctypes.byref(net._nr_cfg)
    assert int(lib.nr_mlp_backward_pipelined(cfg, M)) == 1
    x = (torch.rand(M, 3, device=dev) * 3 - 1.5).contiguous()
    d = torch.nn.functional.normalize(torch.randn(M, 3, device=dev), dim=-1).contiguous()
    flat = net.flat_params()
    packed = net._packed_for_forward()
    rgb = torch.empty(M, 3, device=dev)
    sig = torch.empty(M, 1, device=dev)
    saved = torch.empty(int(lib.nr_mlp_saved_bytes(cfg, M)), device=dev, dtype=torch.uint8)
    st = _hip.stream_ptr()
    call("nr_mlp_forward", cfg, ptr(packed), ptr(flat), ptr(x), ptr(d), M, ptr(rgb), ptr(sig), ptr(saved), st)
    g_rgb = torch.randn(M, 3, device=dev) * 1e-3
    g_sig = torch.randn(M, 1, device=dev) * 1e-3
    ws = torch.zeros(int(lib.nr_mlp_workspace_bytes(cfg, M)), device=dev, dtype=torch.uint8)
    off = int(lib.nr_mlp_pipe_status_offset(cfg, M))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(reps):
        ev0.record()
        call("nr_mlp_backward_dxdw", cfg, ptr(packed), ptr(flat), ptr(x), ptr(d), M, ptr(rgb), ptr(sig), ptr(saved),
             ptr(g_rgb), ptr(g_sig), ptr(None), ptr(None), ptr(ws), st)
        ev1.record()
        torch.cuda.synchronize()
        print(f"rep {r}: dxdw {ev0.elapsed_time(ev1):.3f} ms (events)")
    status = int(ws[off:off + 4].view(torch.int32).item())
    rec = ws[off + 256: off + 256 + 512 * 128].view(torch.int64).view(512, 16).cpu()
    used = rec[:, 13] > 0
    rec = rec[used]
    print(f"status {status}, {int(used.sum())} workgroups")
    t0 = int(rec[:, 0].min())
    by = {}
    for row in rec.tolist():
        kind = row[12] & 0xFF
        stage = (row[12] >> 16) & 0xFFFF
        by.setdefault((stage, kind), []).append(row)
    print("stage kind  start_us(min/max)  end_us(min/max)  cyc/tile  MHz | segments cycles/tile | spins/tile")
    for (stage, kind), rows in sorted(by.items()):
        n = len(rows)
        K = sum(r[13] for r in rows) / n
        starts = [(r[0] - t0) / 100 for r in rows]
        ends = [(r[1] - t0) / 100 for r in rows]
        cyc = [sum(r[2:12]) for r in rows]
        dur = [(r[1] - r[0]) / 100 for r in rows]
        mhz = sum(cyc) / max(1e-9, sum(dur))
        segs = {SEG[i]: sum(r[i] for r in rows) / n / K for i in range(2, 11) if any(r[i] for r in rows)}
        sp = sum(r[14] for r in rows) / n / K
        print(f"{stage:3d} {KIND[kind]:5s} {min(starts):7.1f}/{max(starts):7.1f} {min(ends):8.1f}/{max(ends):8.1f} "
              f"{sum(cyc) / n / K:8.0f} {mhz:6.0f} | " + " ".join(f"{k}={v:.0f}" for k, v in segs.items()) +
              f" | {sp:.2f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 786_432)
