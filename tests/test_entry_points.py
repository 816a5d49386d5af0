"""The reference's command-line entry points on the HIP path: ``python -m
noisy_src.train`` and ``python -m noisy_src.train_pose_opt`` (same flags as
train.py:580-640 / train_pose_opt.py:1057-1190) run a few iterations on a tiny
Blender-layout scene written to a temp dir, and leave the reference's CSV logs."""
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def _scene(root: Path, n_train=3, n_val=1, size=16):
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


def test_train_cli(tmp_path):
    from noisy_src.train import main
    _scene(tmp_path / "data")
    main(["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "128", "--num_iters", "3",
          "--log_every", "1", "--output_dir", str(tmp_path / "out"), "--exp_name", "t", "--precision", "bf16"])
    val = (tmp_path / "out" / "t" / "val_metrics.csv").read_text().splitlines()
    assert val[0] == "iteration,psnr,ssim,mse" and len(val) == 2


def test_train_pose_opt_cli(tmp_path):
    from noisy_src.train_pose_opt import main
    _scene(tmp_path / "data")
    main(["--data_root", str(tmp_path / "data"), "--img_scale", "1.0", "--batch_size", "128", "--num_iters", "4",
          "--pose_opt_delay", "2", "--rotation_noise", "5", "--translation_noise_pct", "5", "--noise_seed", "42",
          "--log_every", "1", "--output_dir", str(tmp_path / "out"), "--device", "cuda"])
    runs = list((tmp_path / "out").iterdir())
    assert len(runs) == 1 and "poseopt_noisyinit_rot5.0deg_trans5.0pct" in runs[0].name
    rows = (runs[0] / "train_metrics.csv").read_text().splitlines()
    assert rows[0] == "iteration,loss,loss_coarse,loss_fine,psnr,learning_rate,time_per_iter,rays_per_sec"
    assert len(rows) == 5
