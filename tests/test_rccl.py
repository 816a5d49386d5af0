"""The data-parallel path over RCCL (backend "nccl") on the GPU box.

The box has one MI355X, and RCCL refuses two ranks on one device, so the group is
world 1 under ``torch.distributed.run --nproc-per-node=1``: the real RCCL communicator
and all-reduce kernels run inside the training step (launched by the MLP backward's
gradient-ready hooks, and captured into the hipGraph of ``GraphedTrainer``).  At world
1 the DP step must equal the plain step bit for bit (tests/rccl_worker.py).  The
multi-rank arithmetic (1/world seed, SUM) is covered by test_distributed_gpu.py (gloo,
two ranks) and test_distributed.py (CPU)."""

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def report(tmp_path_factory):
    out = tmp_path_factory.mktemp("rccl")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    # a fresh child: the worker joins the RCCL group before any GPU call
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                    "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                    str(ROOT / "tests" / "rccl_worker.py"), str(out)], check=True, env=env, timeout=600)
    return json.loads((out / "rccl_report.json").read_text())


def test_rccl_group_and_allreduce(report):
    assert report["backend"] == "nccl" and report["world"] == 1
    assert report["allreduce_ok"]


def test_rccl_train_step_equals_plain(report):
    r = report["train_bf16"]
    assert r["grad_norm"] > 0
    assert r["grads_equal"] and r["losses_equal"] and r["params_equal"], r


def test_rccl_pose_step_equals_plain(report):
    r = report["pose_fp32"]
    assert r["poses_moved"] > 0
    assert r["params_and_poses_equal"], r


def test_rccl_graphed_dp_step(report):
    r = report["graph_bf16"]
    assert r["captured"], r.get("error")
    assert r["losses_equal"] and r["params_equal"], r
    assert r["stale_replay_refused"], r
