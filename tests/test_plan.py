"""The fused-MLP layout plan, checked on the host: the dW jobs' wave shares cover every
parameter's gradient exactly once (tests/native/plan_check.cpp compiles the plan
source robust-nerf_amd/csrc/mlp_plan.cpp.inc with g++; no GPU)."""

import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def plan_check(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path_factory.mktemp("plan") / "plan_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-D__host__=", "-D__device__=", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'robust-nerf_amd' / 'csrc'}", str(ROOT / "tests" / "native" / "plan_check.cpp"),
                    "-o", str(exe)], check=True)
    return exe


# pos_freqs dir_freqs n_layers skip_mask use_view_dirs precision
CONFIGS = [(10, 4, 8, 1 << 4, 1, 1), (10, 4, 8, 1 << 4, 1, 0), (10, 4, 8, 1 << 4, 1, 2), (10, 4, 8, 1 << 4, 0, 1),
           (6, 2, 4, 1 << 1, 1, 1), (10, 4, 12, (1 << 3) | (1 << 7), 1, 1), (4, 1, 1, 0, 1, 1),
           # two and more skips: x-jobs of more than two dz layers exceed the dW staging
           (10, 4, 7, (1 << 2) | (1 << 5), 1, 1), (10, 4, 7, (1 << 2) | (1 << 5), 1, 0),
           (10, 4, 7, (1 << 2) | (1 << 5), 1, 2), (10, 4, 10, 0b10101010, 1, 1), (10, 4, 8, 0b100100, 1, 0)]


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "-".join(map(str, c)))
def test_every_parameter_gradient_written_once(plan_check, cfg):
    r = subprocess.run([str(plan_check), *map(str, cfg)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "unwritten 0 doubly written 0" in r.stdout
    assert "dW workgroup plan bad 0" in r.stdout


def test_too_many_dw_jobs_fails_cleanly(plan_check):
    """16 layers with a skip after every one: more dW jobs than the kernel arguments
    hold -- the plan refuses the config instead of overrunning its job table."""
    r = subprocess.run([str(plan_check), "10", "4", "16", str((1 << 15) - 1), "1", "1"], capture_output=True, text=True)
    assert r.returncode != 0 and "plan fail" in r.stdout, r.stdout
