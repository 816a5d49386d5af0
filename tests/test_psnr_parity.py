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


def test_merge_pools_disjoint_seed_ranges(tmp_path):
    """psnr_parity --merge: two records of one setup with disjoint seeds give the pooled
    paired statistics; a seed present in both is refused."""
    mod = _mod()

    def rec(seeds, path):
        res = [{"impl": i, "precision": p, "seed": s, "test_psnr": 30.0 + s + d, "per_view": None, "iters": 10,
                "batch": 4, "size": 8, "train_seconds": 1.0}
               for s in seeds for (i, p), d in zip(mod.IMPLS, (0.0, 0.1, -0.2))]
        mod.summarize_results(res, 10, 8, 4, None, 250, path)

    rec([0, 1, 2], tmp_path / "a.json")
    rec([3, 4], tmp_path / "b.json")
    mod.merge(tmp_path / "m.json", [tmp_path / "a.json", tmp_path / "b.json"])
    m = json.loads((tmp_path / "m.json").read_text())
    assert m["seeds"] == 5 and m["lr_decay"] == 250
    assert m["delta_vs_ref"]["hip_fp32"]["paired_mean_db"] == pytest.approx(0.1)
    assert m["delta_vs_ref"]["hip_bf16"]["paired_mean_db"] == pytest.approx(-0.2)
    rec([2, 5], tmp_path / "c.json")
    with pytest.raises(SystemExit, match="twice"):
        mod.merge(tmp_path / "x.json", [tmp_path / "a.json", tmp_path / "c.json"])
