"""`python -m noisy_src.train --graph` on the tiny test scene, in a fresh process.
python tools/graph_probe_cli.py OUTDIR [extra train flags...]"""
import sys
from pathlib import Path

sys.path[:0] = [".", "robust-nerf_amd", "tests"]
from test_entry_points import _scene  # noqa: E402
from noisy_src.train import main  # noqa: E402

out = Path(sys.argv[1])
_scene(out / "data")
main(["--data_root", str(out / "data"), "--img_scale", "1.0", "--batch_size", "100", "--num_iters", "10",
      "--val_every", "4", "--save_every", "100", "--output_dir", str(out / "out"), "--exp_name", "g",
      "--precision", "bf16"] + sys.argv[2:])
print("ok", flush=True)
