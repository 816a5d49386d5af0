"""CPU: the bench line's per-kernel table agrees with its headline.

With a committed rocprof summary of the benchmarked sources, every fused-MLP entry takes
its launch time from that summary (``ms_source`` "rocprof"), the dominant entry's MFMA
fraction equals the headline ``roofline.frac`` computed from the same time, and one
step's fused-MLP launches sum to at most the step.  Without one, the entries are labelled
"bracketed" and carry no fraction at all.  Uses the committed round-6 summary and bench
record (profiles/), so it runs without a GPU."""

import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

N_PARAMS = 595_844


def _summary_rows(name="r06_kernel_summary.csv"):
    rows = {}
    with open(ROOT / "profiles" / name) as f:
        for r in csv.DictReader(f):
            if r.get("M_samples") and r.get("precision") in ("bf16", ""):
                rows[(r["kernel"], int(r["M_samples"]))] = r
    return rows


def _wcalls(rows, live_ms=9.0):
    """The bench's warm-up call table for the keys the summary holds (bracketed times
    deliberately far off, so a fallback to them would show)."""
    out = {}
    for entry, kerns in bench.KERNEL_OF.items():
        for (k, M) in rows:
            if k in kerns:
                out[f"{entry}[M={M}]"] = (1, live_ms)
    return out


def test_rocprof_basis_agrees_with_headline():
    rows = _summary_rows()
    ktab, _ = bench.kernel_table(_wcalls(rows), "bf16", N_PARAMS, rp_rows=rows)
    assert ktab and all(v["ms_source"] == "rocprof" for v in ktab.values())
    dw = ktab["nr_mlp_backward_dw[M=786432]"]
    rp_ms = float(rows[("mlp_dw_kernel", 786432)]["timed_avg_ms"])
    assert dw["ms"] == round(rp_ms, 4)
    _, frac, _ = bench.mfma_roofline("nr_mlp_backward_dw", 786432, rp_ms, "bf16")
    assert abs(dw["mfma_frac"] - frac) < 1e-4
    # the dominant entry (largest time) is the headline's kernel
    assert max(ktab, key=lambda k: ktab[k]["ms"]) == "nr_mlp_backward_dw[M=786432]"
    # one step's fused-MLP launches fit in the recorded step of the same tree
    rec = json.loads((ROOT / "profiles" / "r06_bench_full.json").read_text().strip().splitlines()[-1])
    assert sum(v["ms"] for v in ktab.values()) <= rec["ms_per_step"]


def test_committed_summary_covers_every_entry():
    """bench.rocprof_summary picks up every fused-MLP key of the step from the committed
    summary, the precision-independent slab reduction included, when its source hash is
    this tree's."""
    rows, src = bench.rocprof_summary("bf16")
    if src is None:
        import pytest
        pytest.skip("no committed kernel summary of this tree's sources (re-profile after a csrc change)")
    keys = {(k, M) for k, M in rows}
    for entry, kerns in bench.KERNEL_OF.items():
        for M in (262144, 786432):
            assert any((k, M) in keys for k in kerns), (entry, M)


def test_bracketed_entries_carry_no_fraction():
    rows = _summary_rows()
    ktab, _ = bench.kernel_table(_wcalls(rows, live_ms=0.5), "bf16", N_PARAMS, rp_rows=None)
    assert ktab and all(v["ms_source"] == "bracketed" for v in ktab.values())
    for v in ktab.values():
        assert not any(k.endswith("_frac") or k.endswith("tflops") for k in v), v


def test_active_fraction_scales_executed_work():
    """On a skipping backward the dX / dW fractions count the executed tiles only."""
    rows = _summary_rows()
    full, _ = bench.kernel_table(_wcalls(rows), "bf16", N_PARAMS, rp_rows=rows)
    part, _ = bench.kernel_table(_wcalls(rows), "bf16", N_PARAMS, rp_rows=rows, active={786432: 0.37})
    k = "nr_mlp_backward_dw[M=786432]"
    assert abs(part[k]["mfma_frac"] - 0.37 * full[k]["mfma_frac"]) < 1e-3
    f = "nr_mlp_forward[M=786432]"
    assert part[f]["mfma_frac"] == full[f]["mfma_frac"]  # the forward never skips
