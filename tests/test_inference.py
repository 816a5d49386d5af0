"""Checkpoint format and the sharded test-set evaluation.

CPU side: the reference's checkpoint keys / file names round-trip through
``torch.load(weights_only=True)``; ``evaluate_test_set`` sharded over two gloo ranks
returns the same per-image records and summary as one process (rendering replaced by
a deterministic stand-in: the sharding, noise draws, gather and files are what is
under test).  The GPU test renders through the HIP path."""

import json
import os
import socket
from dataclasses import dataclass

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from noisy_src import inference
from noisy_src.config import NeRFConfig
from noisy_src.data import BlenderData
from noisy_src.noise import NoiseConfig


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_checkpoint_round_trip(tmp_path):
    from noisy_src.model import create_nerf
    from noisy_src.train import load_checkpoint, save_checkpoint
    cfg = NeRFConfig()
    torch.manual_seed(0)
    mc, mf = create_nerf(cfg.model)
    opt = torch.optim.Adam(list(mc.parameters()) + list(mf.parameters()), lr=5e-4)
    save_checkpoint(tmp_path, 1234, mc, mf, opt, cfg, noise_config=NoiseConfig(rotation_noise_deg=5.0),
                    metrics={"psnr": 25.0}, is_best=True)
    for name in ("checkpoint_0001234.pt", "checkpoint_latest.pt", "checkpoint_best.pt"):
        assert (tmp_path / name).exists()
    ck = torch.load(tmp_path / "checkpoint_latest.pt", weights_only=True)
    assert set(ck) == {"iteration", "model_coarse", "model_fine", "optimizer", "config", "metrics", "noise_config",
                       "mi355x"}
    assert list(ck["model_coarse"]) == list(mc.state_dict())  # nn.Linear naming of the reference
    renderer, c, it = inference.load_checkpoint(tmp_path / "checkpoint_latest.pt", device="cpu")
    assert it == 1234 and c["model"]["hidden_dim"] == 256 and c["render"]["num_samples_fine"] == 128
    for a, b in ((renderer.model_coarse, mc), (renderer.model_fine, mf)):
        sa, sb = a.state_dict(), b.state_dict()
        assert all(torch.equal(sa[k], sb[k]) for k in sb)
    torch.manual_seed(1)
    mc2, mf2 = create_nerf(cfg.model)
    opt2 = torch.optim.Adam(list(mc2.parameters()) + list(mf2.parameters()), lr=5e-4)
    assert load_checkpoint(tmp_path / "checkpoint_0001234.pt", mc2, mf2, opt2) == 1234
    s2, s1 = mc2.state_dict(), mc.state_dict()
    assert all(torch.equal(s2[k], s1[k]) for k in s1)
    assert opt2.state_dict()["param_groups"][0]["lr"] == 5e-4


@dataclass
class _RefModelConfig:
    """The reference's ModelConfig fields only (noisy_src/config.py:10-24)."""

    pos_freqs: int = 10
    dir_freqs: int = 4
    hidden_dim: int = 256
    num_hidden_layers: int = 8
    skips: tuple = (4,)
    use_view_dirs: bool = True


def test_checkpoint_readable_by_reference_loaders(tmp_path):
    """A checkpoint written from FusedAdam loads where the reference loads it: its
    ``ModelConfig(**cfg["model"])`` (inference.py:53) and a plain ``torch.optim.Adam``
    whose ``step()`` reads every Adam param-group key."""
    from noisy_src.model import create_nerf
    from noisy_src.optim import FusedAdam
    from noisy_src.train import save_checkpoint
    cfg = NeRFConfig()
    cfg.model.precision = "bf16"
    torch.manual_seed(0)
    mc, mf = create_nerf(cfg.model)
    fused = FusedAdam(list(mc.parameters()) + list(mf.parameters()), lr=5e-4)
    save_checkpoint(tmp_path, 7, mc, mf, fused, cfg)
    ck = torch.load(tmp_path / "checkpoint_latest.pt", weights_only=True)
    _RefModelConfig(**ck["config"]["model"])  # no unexpected keyword
    assert ck["mi355x"]["precision"] == "bf16"
    renderer, _, _ = inference.load_checkpoint(tmp_path / "checkpoint_latest.pt", device="cpu")
    assert renderer.model_coarse.config.precision == "bf16"
    torch.manual_seed(1)
    a, b = create_nerf(cfg.model)
    params = list(a.parameters()) + list(b.parameters())
    adam = torch.optim.Adam(params, lr=1.0)
    adam.load_state_dict(ck["optimizer"])
    assert adam.param_groups[0]["lr"] == 5e-4
    for p in params:
        p.grad = torch.ones_like(p)
    adam.step()  # KeyError on a missing param-group key would surface here


def test_fused_adam_rejects_unsupported_options():
    from noisy_src.optim import FusedAdam
    p = [torch.nn.Parameter(torch.zeros(4))]
    with pytest.raises(ValueError):
        FusedAdam(p, weight_decay=0.1)
    with pytest.raises(ValueError):
        FusedAdam(p, amsgrad=True)


def _fake_render(renderer, pose, H, W, focal, chunk_size=4096):
    """Deterministic stand-in for the HIP render: a function of the pose only."""
    base = torch.sigmoid(pose[:3, :].sum(0)[:3])
    img = base.view(1, 1, 3).expand(H, W, 3).clone()
    img[::2] *= 0.9
    return {"rgb": img, "depth": torch.linspace(2, 6, H * W).view(H, W), "acc": torch.ones(H, W)}


def _scene():
    g = torch.Generator().manual_seed(7)
    poses = torch.eye(4).repeat(5, 1, 1)
    poses[:, :3, 3] = torch.randn(5, 3, generator=g) * 4
    return BlenderData(images=torch.rand(5, 8, 6, 3, generator=g), poses=poses, H=8, W=6, focal=7.0)


def _eval_worker(rank, world, port, outdir, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        inference.render_image = _fake_render
        res = inference.evaluate_test_set(None, _scene(), outdir, NoiseConfig(rotation_noise_deg=2.0,
                                          translation_noise=0.05, seed=3), device="cpu",
                                          process_group=dist.group.WORLD, log=lambda *_: None)
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_evaluate_test_set_sharded_matches_single(tmp_path, monkeypatch):
    monkeypatch.setattr(inference, "render_image", _fake_render)
    noise = NoiseConfig(rotation_noise_deg=2.0, translation_noise=0.05, seed=3)
    one = inference.evaluate_test_set(None, _scene(), tmp_path / "one", noise, device="cpu", log=lambda *_: None)
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_eval_worker, args=(2, _free_port(), str(tmp_path / "two"), out), nprocs=2, join=True)
        res = dict(out)
    assert res[0] == res[1]
    for k in ("psnr_mean", "ssim_mean", "mse_mean", "n_images"):
        assert res[0][k] == pytest.approx(one[k], rel=1e-12), k
    assert res[0]["actual_noise"] == pytest.approx(one["actual_noise"])
    a = json.loads((tmp_path / "one" / "per_image_metrics.json").read_text())
    b = json.loads((tmp_path / "two" / "per_image_metrics.json").read_text())
    assert [r["image"] for r in b] == list(range(5))
    for ra, rb in zip(a, b):
        assert ra["psnr"] == pytest.approx(rb["psnr"]) and ra["noise_rotation_error_deg"] == pytest.approx(
            rb["noise_rotation_error_deg"])
    # every view's images were written by the rank that rendered it
    assert all((tmp_path / "two" / f"pred_{i:03d}.png").exists() for i in range(5))


@pytest.mark.gpu
def test_evaluate_test_set_gpu(tmp_path):
    """Rendering through the HIP path: per-image PSNR equals compute_psnr of render_image."""
    import numpy as np
    from pathlib import Path

    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.data import synthetic_blender_data
    from noisy_src.metrics import compute_psnr
    from noisy_src.model import create_nerf
    from noisy_src.rendering import NeRFRenderer
    from noisy_src.train import render_image
    golden = Path(__file__).resolve().parent / "golden"
    poses = torch.from_numpy(np.load(sorted(golden.glob("final_poses_*.npz"))[0])["ground_truth_poses"][:3])
    data = synthetic_blender_data(poses, H=16, W=16, device="cuda")
    torch.manual_seed(0)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    renderer = NeRFRenderer(mc.cuda(), mf.cuda(), RenderConfig())
    res = inference.evaluate_test_set(renderer, data, tmp_path, NoiseConfig(), device="cuda", log=lambda *_: None)
    want = [compute_psnr(render_image(renderer, data.poses[i], 16, 16, data.focal)["rgb"], data.images[i]).item()
            for i in range(3)]
    assert res["psnr_mean"] == pytest.approx(sum(want) / 3, abs=1e-5)
    assert res["n_images"] == 3 and (tmp_path / "test_metrics.json").exists()
