"""Per-step overlap of the data-parallel gradient all-reduce with the backward, from a
rocprofv3 kernel trace of ``bench.py --dp`` (the fine network's all-reduce
is issued as soon as its gradient is reduced and runs while the coarse backward still
computes).

    python tools/overlap_trace.py gpurun_out/prof_dp [out.txt]

Steps are delimited by ``adam_multi_kernel``.  For every step the script lists, relative
to the step's first kernel: the fine gradient's slab reduction end, each RCCL kernel
(start / end), and the coarse backward's dX / dW / reduction kernels; it then states
whether the first RCCL kernel started before the coarse dW kernel ended.
"""

from __future__ import annotations

import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from prof_summary import MTracker, short  # noqa: E402


def main(trace_dir: str, out: str | None = None) -> None:
    with open(Path(trace_dir) / "run_kernel_trace.csv") as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    track = MTracker()
    recs = []
    # M attribution needs dispatch order (stream order); timestamps give overlap
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        M = track(r["Kernel_Name"], grid)
        recs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], M))
    recs.sort()
    ends = [i for i, x in enumerate(recs) if short(x[2]) == "adam_multi_kernel"]
    lines, n_overlap, n_steps = [], 0, 0
    Ms = sorted({x[3] for x in recs if x[3]})
    m_coarse, m_fine = (Ms[0], Ms[-1]) if len(Ms) >= 2 else (None, None)
    for a, b in zip(ends, ends[1:]):
        step = recs[a + 1:b + 1]
        t0 = step[0][0]
        rccl = [x for x in step if "nccl" in x[2].lower()]
        red_f = [x for x in step if short(x[2]) == "mlp_dw_reduce_kernel" and x[3] == m_fine]
        co = [x for x in step if x[3] == m_coarse and short(x[2]) in ("mlp_bwd_rbm_kernel", "mlp_dw_kernel",
                                                                         "mlp_dw_reduce_kernel")]
        if not rccl or not red_f or not co:
            continue
        n_steps += 1
        dw_c = [x for x in co if short(x[2]) == "mlp_dw_kernel"]
        overlap = bool(dw_c) and rccl[0][0] < dw_c[-1][1]
        n_overlap += overlap
        lines.append(f"step {n_steps}: fine reduce ends {(red_f[-1][1] - t0) / 1e3:8.1f} us; "
                     + "; ".join(f"{'RCCL' if 'nccl' in x[2].lower() else short(x[2])}[M={x[3] or '-'}] "
                                 f"{(x[0] - t0) / 1e3:.1f}-{(x[1] - t0) / 1e3:.1f}"
                                 for x in sorted(rccl + co))
                     + f"; first all-reduce kernel starts before the coarse dW ends: {overlap}")
    if not any("nccl" in x[2].lower() for x in recs):
        lines.append("no RCCL kernel in this trace: a one-rank communicator completes an all-reduce without "
                     "launching one, so the overlap shows only in a multi-rank run (bench.py's topology "
                     "fields time the all-reduce with HIP events at any world size)")
    lines.append(f"{n_overlap} of {n_steps} steps: the first RCCL kernel starts before the coarse backward's dW "
                 f"kernel ends (coarse M={m_coarse}, fine M={m_fine})")
    text = "\n".join(lines)
    print(text)
    if out:
        Path(out).write_text(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
