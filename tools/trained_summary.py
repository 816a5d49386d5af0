"""Per-phase kernel times of bench.py's trained-state leg from a rocprofv3 kernel trace.

    python tools/trained_summary.py TRACE_DIR [out.txt]

The leg runs skip / dense / skip, each 3 + 4 + 50 steps (bench.trained_state_leg); the
fused-MLP launches of the last 3 x 57 steps are those runs, and the last 50 of each run
are its timed steps.  Prints, per run and kernel (grid), the median launch time."""

from __future__ import annotations

import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

RUN, TIMED = 57, 50
KERNELS = ("mlp_fwd_rbm_kernel", "mlp_bwd_rbm_kernel", "mlp_dw_kernel", "tile_flags_kernel")


def main(trace_dir: str, out: str | None = None) -> None:
    with open(Path(trace_dir) / "run_kernel_trace.csv") as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    seq = defaultdict(list)  # (kernel, grid) -> durations in launch order
    last_dx = 0  # dW's grid is the same for both nets: tag it with the dX launch before it
    for r in rows:
        name = r["Kernel_Name"]
        k = next((k for k in KERNELS if k in name), None)
        if k is None:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        if k == "mlp_bwd_rbm_kernel":
            last_dx = grid
        if k == "mlp_dw_kernel":
            grid = last_dx  # shown under the dX grid of its net
        seq[(k, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = ["# trained-state leg (bench.py), median launch time per timed run, us (rocprofv3 kernel trace);",
             "# grid = threads of the launch (dW: of its net's dX launch); the 1,024-ray training launches are left out",
             f"{'kernel':22s} {'grid':>9s} {'skip_a':>8s} {'dense':>8s} {'skip_b':>8s}"]
    for (k, g), v in sorted(seq.items()):
        # the leg's 4,096-ray launches only (the 1,024-ray training's are smaller)
        if len(v) < 3 * RUN or g < (32768 if k == "tile_flags_kernel" else 524288):
            continue
        last = v[-3 * RUN:]
        med = [statistics.median(last[i * RUN + RUN - TIMED:(i + 1) * RUN]) for i in range(3)]
        lines.append(f"{k:22s} {g:9d} " + " ".join(f"{m:8.1f}" for m in med))
    text = "\n".join(lines)
    print(text)
    if out:
        Path(out).write_text(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
