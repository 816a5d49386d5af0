"""The reference's command-line entry points on the HIP path: ``python -m noisy_src.train``
and ``python -m noisy_src.train_pose_opt`` (same flags as train.py:580-657 /
train_pose_opt.py:1057-1142) run a few iterations on a tiny Blender-layout scene written
to a temp dir.  Their output folders are checked against the layout of the reference's
own recorded runs (tests/golden/reference_artifacts.json "layout", extracted from
/root/reference/outputs by tests/golden/make_fixtures.py): files, CSV headers and rows,
JSON key sets, image names, checkpoint keys and the final_poses.pt keys.  The
data-parallel mode runs both CLIs under torch.distributed.run with two ranks."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
LAYOUT = json.loads((GOLDEN / "reference_artifacts.json").read_text())["layout"]


def _scene(root: Path, n_train=3, n_val=2, size=16):
    from PIL import Image
    poses = np.load(sorted(GOLDEN.glob("final_poses_*.npz"))[0])["ground_truth_poses"]
    scene = root / "lego"
    rng = np.random.default_rng(0)
    for split, n in (("train", n_train), ("val", n_val)):
        (scene / split).mkdir(parents=True, exist_ok=True)
        frames = []
        for i in range(n):
            Image.fromarray(rng.integers(0, 256, (size, size, 4), dtype=np.uint8), "RGBA").save(
                scene / split / f"r_{i}.png")
            frames.append({"file_path": f"./{split}/r_{i}", "transform_matrix": poses[i].tolist()})
        (scene / f"transforms_{split}.json").write_text(json.dumps({"camera_angle_x": 0.6911112, "frames": frames}))


def _check_layout(run: Path, kind: str, n_iters: int, ckpt_iters):
    lay = LAYOUT[kind]
    got_top = sorted(f.name for f in run.iterdir())
    for f in lay["top_files"]:
        assert f in got_top, (f, got_top)
    for f in lay["log_files"]:
        head = (run / "logs" / f).read_text().splitlines()[0]
        assert head == lay["csv_headers"][f], (f, head)
    rows = (run / "logs" / "train_metrics.csv").read_text().splitlines()
    assert len(rows) == 1 + n_iters
    for name, key in (("summary.json", "summary_keys"), ("experiment_config.json", "experiment_config_keys"),
                      ("config.json", "config_keys")):
        have = set(json.loads((run / name).read_text()))
        assert set(lay[key]) <= have, (name, set(lay[key]) - have)
    summ = json.loads((run / "summary.json").read_text())
    assert summ["model_coarse_total_params"] == 595844 and summ["total_iterations"] == n_iters
    for pat in lay["image_patterns"]:
        assert (run / "images" / pat.format(i=0, it=n_iters)).exists(), pat
    for it in ckpt_iters:
        assert (run / f"checkpoint_{it:07d}.pt").exists(), it
    assert (run / "checkpoint_latest.pt").exists()
    ck = torch.load(run / "checkpoint_latest.pt", weights_only=True, map_location="cpu")
    assert "precision" not in ck["config"]["model"]  # the reference's ModelConfig(**cfg["model"]) loads it
    return ck


def test_train_cli(tmp_path):
    from noisy_src import inference
    from noisy_src.train import main
    _scene(tmp_path / "data")
    main(["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "128", "--num_iters", "5",
          "--log_every", "1", "--val_every", "2", "--save_every", "3", "--output_dir", str(tmp_path / "out"),
          "--exp_name", "t", "--precision", "bf16", "--rotation_noise", "1.0", "--noise_seed", "3"])
    run = tmp_path / "out" / "t"
    ck = _check_layout(run, "train", 5, ckpt_iters=(2, 3, 4, 5))
    assert set(ck) >= {"iteration", "model_coarse", "model_fine", "optimizer", "config", "noise_config"}
    assert ck["noise_config"]["rotation_noise_deg"] == 1.0 and ck["iteration"] == 5
    assert (run / "checkpoint_best.pt").exists()
    val = (run / "logs" / "val_metrics.csv").read_text().splitlines()
    assert [r.split(",")[0] for r in val[1:]] == ["2", "4", "5"]  # val_every 2, then the final evaluation
    exp = json.loads((run / "experiment_config.json").read_text())
    assert exp["noise_config"]["has_noise"] and exp["noise_config"]["rotation_noise_deg"] == 1.0
    renderer, cfg, it = inference.load_checkpoint(run / "checkpoint_latest.pt", device="cuda")
    assert it == 5 and renderer.model_coarse.config.precision == "bf16"


def test_train_cli_coarse_only(tmp_path):
    """BASELINE cfg #1 shape (--no_hierarchical): no fine network anywhere (train.py:382-387)."""
    from noisy_src.train import main
    _scene(tmp_path / "data")
    main(["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "64", "--num_iters", "2",
          "--no_hierarchical", "--output_dir", str(tmp_path / "out"), "--exp_name", "c"])
    ck = torch.load(tmp_path / "out" / "c" / "checkpoint_latest.pt", weights_only=True, map_location="cpu")
    assert "model_fine" not in ck
    summ = json.loads((tmp_path / "out" / "c" / "summary.json").read_text())
    assert "model_fine_total_params" not in summ
    head = (tmp_path / "out" / "c" / "logs" / "train_metrics.csv").read_text().splitlines()[0]
    assert head == "iteration,loss,loss_coarse,psnr,learning_rate,time_per_iter,rays_per_sec"


def test_train_cli_graph_matches_eager(tmp_path):
    """``--graph``: iteration 0 eager, then the step replayed from a hipGraph; an epoch's
    short final batch (768 rays / 100) runs eagerly between replays, and validation runs
    mid-way.  The weights and every logged loss equal the eager run's bit for bit."""
    from noisy_src.train import main
    _scene(tmp_path / "data")
    cks, rows = {}, {}
    for name, extra in (("e", []), ("g", ["--graph"])):
        main(["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "100", "--num_iters", "10",
              "--val_every", "4", "--save_every", "100", "--output_dir", str(tmp_path / "out"), "--exp_name", name,
              "--precision", "bf16"] + extra)
        run = tmp_path / "out" / name
        cks[name] = torch.load(run / "checkpoint_latest.pt", weights_only=True, map_location="cpu")
        rows[name] = [r.split(",")[:3] for r in (run / "logs" / "train_metrics.csv").read_text().splitlines()]
    assert len(rows["g"]) == 11 and rows["g"] == rows["e"]
    for net in ("model_coarse", "model_fine"):
        for k, v in cks["e"][net].items():
            assert torch.equal(v, cks["g"][net][k]), (net, k)
    for k, v in cks["e"]["optimizer"]["state"].items():
        assert torch.equal(v["exp_avg"], cks["g"]["optimizer"]["state"][k]["exp_avg"]), k


def test_train_pose_opt_cli(tmp_path):
    from noisy_src.train_pose_opt import main
    _scene(tmp_path / "data")
    main(["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "128", "--num_iters", "4",
          "--pose_opt_delay", "2", "--rotation_noise", "5", "--translation_noise_pct", "5", "--noise_seed", "42",
          "--log_every", "1", "--val_every", "2", "--output_dir", str(tmp_path / "out"), "--device", "cuda"])
    runs = list((tmp_path / "out").iterdir())
    assert len(runs) == 1 and "poseopt_noisyinit_rot5.0deg_trans5.0pct" in runs[0].name
    ck = _check_layout(runs[0], "pose_opt", 4, ckpt_iters=(2, 4))
    assert set(ck) >= {"iteration", "model_coarse", "model_fine", "camera_params", "optimizer_nerf",
                       "optimizer_poses", "initial_poses", "config", "pose_errors", "noise_config"}
    fp = torch.load(runs[0] / "final_poses.pt", weights_only=True)
    assert list(fp) == LAYOUT["pose_opt"]["final_poses_keys"]
    init, opt, gt = fp["initial_poses"], fp["optimized_poses"], fp["ground_truth_poses"]
    assert init.shape == opt.shape == gt.shape == (3, 4, 4)
    # the reference's dead rotation gradient: R never moves, t does
    assert torch.equal(opt[:, :3, :3], init[:, :3, :3])
    assert (opt[:, :3, 3] - init[:, :3, 3]).abs().max() > 0
    val = (runs[0] / "logs" / "val_metrics.csv").read_text().splitlines()
    assert len(val) == 2  # the final evaluation is not CSV-logged (train_pose_opt.py:1002-1019)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("module", ["noisy_src.train", "noisy_src.train_pose_opt"])
def test_cli_data_parallel_two_ranks(tmp_path, module):
    """torchrun mode of both CLIs: one process per rank, the global batch sliced, the
    gradients averaged (gloo here: the two ranks share one GPU and RCCL refuses that).
    Rank 0 alone writes the run folder; its final weights equal the one-process run
    trained on the same global batches (to fp32 summation order)."""
    _scene(tmp_path / "data")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", NR_DIST_BACKEND="gloo",
               PYTHONPATH=os.pathsep.join([str(ROOT / "robust-nerf_amd"), os.environ.get("PYTHONPATH", "")]))
    args = ["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "128", "--num_iters", "3",
            "--val_every", "100"]
    if module.endswith("pose_opt"):
        args += ["--pose_opt_delay", "1", "--translation_noise_pct", "5", "--noise_seed", "1"]
    else:
        args += ["--exp_name", "dp"]
    outs = {}
    for world in (1, 2):
        out = tmp_path / f"out{world}"
        launch = [sys.executable, "-m", module] if world == 1 else [
            sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
            "127.0.0.1", "--master-port", str(_free_port()), "-m", module]
        subprocess.run(launch + args + ["--output_dir", str(out)], check=True, env=env, timeout=600, cwd=str(ROOT))
        runs = list(out.iterdir())
        assert len(runs) == 1
        outs[world] = torch.load(runs[0] / "checkpoint_latest.pt", weights_only=True, map_location="cpu")
    a, b = outs[1]["model_fine"], outs[2]["model_fine"]
    for k in a:
        # Adam moves a coordinate by ~lr*sign(g) per step; coordinates with ~0 gradient can
        # flip under a different summation order
        assert (a[k] - b[k]).abs().max() < 2 * 3 * 5e-4, k
    frac = np.mean([((a[k] - b[k]).abs() < 1e-5).float().mean().item() for k in a])
    assert frac > 0.95
