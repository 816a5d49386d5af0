"""Summarise a rocprofv3 run for profiles/: per-(kernel, grid) launch durations
from the kernel trace, and HBM traffic per launch from the two PMC passes.

    python tools/prof_summary.py gpurun_out ROUND_TAG

reads  gpurun_out/prof/run_kernel_trace.csv
       gpurun_out/pmc_fetch/run_counter_collection.csv   (FETCH_SIZE, KB)
       gpurun_out/pmc_write/run_counter_collection.csv   (WRITE_SIZE, KB)
writes profiles/<tag>_kernel_summary.csv and profiles/traffic.json.

Traffic = 2 x FETCH_SIZE + WRITE_SIZE: on gfx950 FETCH_SIZE counts exactly half of
the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section),
WRITE_SIZE counts 16-B streaming stores exactly.  Both count Infinity-Cache hits.
"""

from __future__ import annotations

import csv
import hashlib
import json
import re
import statistics
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

# fused-MLP grid size (workgroups x threads) -> samples M, per kernel family
FAMILIES = {"mlp_fwd_kernel": "nr_mlp_forward", "mlp_bwd_kernel": "nr_mlp_backward_dx",
            "mlp_fwd_rbm_kernel": "nr_mlp_forward", "mlp_bwd_rbm_kernel": "nr_mlp_backward_dx",
            "mlp_dinput_kernel": "nr_mlp_backward_dx (input grads)",
            "mlp_dw_kernel": "nr_mlp_backward_dw", "mlp_dw_reduce_kernel": "nr_mlp_backward_reduce"}


def source_hash() -> str:
    """sha1 over the HIP sources and the ABI header (bench.py computes the same hash, so
    it uses a kernel summary only when it was profiled from the benchmarked sources);
    NR_SOURCE_HASH overrides it when re-summarising a trace taken from an older tree, and
    every row it writes then says so (``hash_overridden``, which bench.py refuses)."""
    import os
    if os.environ.get("NR_SOURCE_HASH"):
        return os.environ["NR_SOURCE_HASH"]
    return computed_hash()


def computed_hash() -> str:
    h = hashlib.sha1()
    files = sorted((ROOT / "robust-nerf_amd" / "csrc").glob("*")) + [ROOT / "include" / "nerf_hip.h"]
    for f in files:
        if f.suffix in (".hip", ".inc", ".hpp", ".h"):
            h.update(f.name.encode())
            h.update(f.read_bytes())
    return h.hexdigest()[:12]


def short(name: str) -> str:
    m = re.search(r"nr::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def precision_of(name: str) -> str:
    m = re.search(r"nr::mlp_\w+_kernel<(\d)", name)
    return {"1": "bf16", "0": "fp32", "2": "fp16"}.get(m.group(1), "") if m else ""


def is_training_forward(name: str) -> bool:
    """A forward launch that saves activations (TRAIN template flag) and so has exactly
    one backward launch later in the step."""
    return short(name) in ("mlp_fwd_kernel", "mlp_fwd_rbm_kernel") and "true" in name.split("(")[0]


class MTracker:
    """M of every fused-MLP launch in stream order.  The forward kernels run one
    32-sample tile per wave, so their grid gives M (rounded up to whole workgroups).  A
    dX launch takes the M of the newest training forward not yet matched (autograd runs
    the backwards in reverse forward order; its grid covers whole 256-tile segments, so
    it gives M only rounded up to 8,192 samples).  dW, its reduction and the input
    gradients follow the backward launch of the same M."""

    def __init__(self):
        self.last = 0
        self.fwd_stack = []

    def __call__(self, name: str, grid: int) -> int:
        fam = short(name)
        M = 0
        if fam in ("mlp_fwd_kernel", "mlp_fwd_rbm_kernel"):
            M = grid // 64 * 32
            if is_training_forward(name):
                self.fwd_stack.append(M)
        elif fam in ("mlp_bwd_kernel", "mlp_bwd_rbm_kernel"):
            M = self.fwd_stack.pop() if self.fwd_stack else grid // 64 * 32
        elif fam in ("mlp_dw_kernel", "mlp_dw_reduce_kernel", "mlp_dinput_kernel"):
            M = self.last
        self.last = M or self.last
        return M


def main(out_dir: str, tag: str, timed_steps: int = 0) -> None:
    """``timed_steps`` K: also average each fused-MLP key over its last K launches, the
    launches of bench.py's timed region (each key launches once per step)."""
    base = Path(out_dir)
    rows = defaultdict(list)
    with open(base / "prof" / "run_kernel_trace.csv") as f:
        trace = sorted(csv.DictReader(f), key=lambda r: int(r["Dispatch_Id"]))
    track = MTracker()
    for r in trace:
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        M = track(r["Kernel_Name"], grid)
        rows[(r["Kernel_Name"], grid, M)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    summ = ROOT / "profiles" / f"{tag}_kernel_summary.csv"
    with open(summ, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "precision", "grid_threads", "M_samples", "calls", "avg_ms", "median_ms", "total_ms",
                    "timed_avg_ms", "source_hash", "hash_overridden"])
        sh = source_hash()
        over = "" if sh == computed_hash() else f"computed {computed_hash()}"
        for (k, g, M), v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
            timed = v[-timed_steps:] if (timed_steps and M and len(v) >= timed_steps) else []
            w.writerow([short(k), precision_of(k), g, M or "", len(v), f"{statistics.mean(v):.4f}",
                        f"{statistics.median(v):.4f}", f"{sum(v):.3f}",
                        f"{statistics.mean(timed):.4f}" if timed else "", sh, over])
    print(f"wrote {summ}")

    counters = defaultdict(lambda: defaultdict(list))
    for sub, cname in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        p = base / sub / "run_counter_collection.csv"
        if not p.exists():
            continue
        with open(p) as f:
            recs_ = sorted((r for r in csv.DictReader(f) if r["Counter_Name"] == cname),
                           key=lambda r: int(r["Dispatch_Id"]))
        track = MTracker()
        for r in recs_:
            M = track(r["Kernel_Name"], int(r["Grid_Size"]))
            key = (r["Kernel_Name"], M)
            counters[key][cname].append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
    recs = []
    for (k, M), c in sorted(counters.items()):
        fam = short(k)
        if fam not in FAMILIES or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        fetch = statistics.median(c["FETCH_SIZE"])
        write = statistics.median(c["WRITE_SIZE"])
        recs.append({"kernel": fam, "entry": FAMILIES[fam], "precision": precision_of(k), "M": M,
                     "fetch_size_bytes": fetch, "write_size_bytes": write,
                     "bytes_per_launch": 2.0 * fetch + write, "launches": len(c["FETCH_SIZE"])})
    if not recs:
        print("no PMC passes under", base, "- profiles/traffic.json left as it is")
        return
    out = {"source_hash": source_hash(),
           **({"hash_overridden": f"computed {computed_hash()}"} if source_hash() != computed_hash() else {}),
           "source": f"profiles/{tag}: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                     "python bench.py --steps 2 --warmup 1 --no-cpu-baseline; traffic = 2*FETCH_SIZE + WRITE_SIZE per launch (median)",
           "kernels": recs,
           # each (kernel, M) launches once per training step: the step's MLP HBM bytes
           "per_step_mlp_bytes": sum(r["bytes_per_launch"] for r in recs)}
    (ROOT / "profiles" / "traffic.json").write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 0)
