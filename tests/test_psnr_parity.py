"""Test-PSNR parity at equal iterations (BASELINE metric, second half) on the analytic
scene of tests/psnr_parity.py, in a short configuration; the full multi-seed run
(`python tests/psnr_parity.py`) is recorded in profiles/r01_psnr_parity.json."""
import importlib.util
import pathlib

import pytest

pytestmark = pytest.mark.gpu


def _mod():
    spec = importlib.util.spec_from_file_location("psnr_parity", pathlib.Path(__file__).parent / "psnr_parity.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


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
    # in profiles/r01_psnr_parity.json.
    assert abs(hip - ref) < 1.0, (hip, ref)
    assert abs(bf - ref) < 1.0, (bf, ref)
