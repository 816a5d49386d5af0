"""One training step's kernel timeline from a rocprofv3 kernel trace (bench.py).

    python tools/step_timeline.py gpurun_out/prof [step_index_from_end=2] [out.txt]

Steps are delimited by ``adam_multi_kernel``; times are in microseconds from the end
of the previous step's Adam launch, with each kernel's hardware queue.  Also prints the
step's wall time and the summed kernel time per queue.
"""

from __future__ import annotations

import csv
import sys
from collections import defaultdict
from pathlib import Path


def main(trace_dir: str, back: int = 2, out: str | None = None) -> None:
    with open(Path(trace_dir) / "run_kernel_trace.csv") as f:
        rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_multi_kernel" in r["Kernel_Name"]]
    a, b = ends[-1 - back], ends[-back]
    t0 = int(rows[a]["End_Timestamp"])
    lines = []
    busy = defaultdict(float)
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id", "?")
        busy[q] += (e - s) / 1e3
        name = r["Kernel_Name"].replace("void ", "")[:60]
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        lines.append(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q={q:>2} {name} grid={g}")
    wall = (int(rows[b]["End_Timestamp"]) - t0) / 1e3
    lines.append(f"step wall {wall:.1f} us; kernel time per queue: "
                 + ", ".join(f"q{q} {v:.1f} us" for q, v in sorted(busy.items())))
    text = "\n".join(lines)
    print(text)
    if out:
        Path(out).write_text(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2, sys.argv[3] if len(sys.argv) > 3 else None)
