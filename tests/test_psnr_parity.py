"""Test-PSNR parity at equal iterations (BASELINE metric, second half) on the analytic
scene of tests/psnr_parity.py: a short GPU configuration (smoke level: two seeds cannot
resolve 0.1 dB), and the check that the committed multi-seed record
(profiles/r02_psnr_parity.json: 20 paired seeds, LR annealed 100x over 2000 iterations)
meets the north-star bar |delta| <= 0.1 dB at ~95 % confidence."""
import importlib.util
import json
import pathlib

import pytest




def _mod():
    spec = importlib.util.spec_from_file_location("psnr_parity", pathlib.Path(__file__).parent / "psnr_parity.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.gpu
def test_psnr_parity_short():
    run = _mod().run
    kw = dict(iters=300, size=32, batch=512)

    def mean_psnr(impl, prec):
        return sum(run(impl, prec, seed=s, **kw)["test_psnr"] for s in (0, 1)) / 2

    ref, hip, bf = mean_psnr("ref", "fp32"), mean_psnr("hip", "fp32"), mean_psnr("hip", "bf16")
    assert ref > 15.0  # it does learn the scene
    # Training is chaotic (a 1-ulp difference flips Adam's step on ~0 gradients), so two
    # seeds per implementation bound the gap only loosely (the reference's own single-run
    # seed-to-seed spread here is ~1 dB); the tighter multi-seed comparison is the long run
    # in profiles/r02_psnr_parity.json (test_recorded_psnr_parity_meets_the_bar).
    assert abs(hip - ref) < 1.0, (hip, ref)
    assert abs(bf - ref) < 1.0, (bf, ref)


@pytest.mark.parametrize("impl", ["hip_fp32", "hip_bf16"])
def test_recorded_psnr_parity_meets_the_bar(impl):
    """The committed record: paired test-PSNR difference to the reference algorithm (the
    oracle, torch fp32) within 0.1 dB at two standard errors, over >= 16 paired seeds."""
    rec = json.loads((pathlib.Path(__file__).resolve().parents[1] / "profiles" / "r02_psnr_parity.json").read_text())
    assert rec["seeds"] >= 16 and rec["iters"] == 2000
    d = rec["delta_vs_ref"][impl]
    assert abs(d["paired_mean_db"]) + 2 * d["paired_se_db"] <= 0.11, d
    assert d["paired_se_db"] <= 0.05, d
