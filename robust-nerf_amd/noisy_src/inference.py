"""
Test-set evaluation and checkpoint loading — drop-in for ShawnnnLiu/Robust-NeRF
``noisy_src/inference.py`` (the eval half of BASELINE.json's metric).

``evaluate_test_set`` keeps the reference's signature, per-image metrics and output
files (inference.py:145-318), with the rendering on the HIP forward-only path
(``render_image`` -> NeRFRenderer, is_train=False) and, given a process group, the
test views sharded across ranks (SURVEY.md §8e "Eval"): rank r renders views
r, r+N, r+2N, ...; the per-image metric records are all-gathered so every rank
returns the same summary, and rank 0 writes the JSON files.  Camera noise is drawn
for every view up front, in view order, from the same seed on every rank (the
reference draws it inside its loop, in the same order; rendering itself draws
nothing), so the noisy poses match the reference's sequential run.
"""

from __future__ import annotations

import json
import time
from datetime import datetime
from pathlib import Path
from typing import Dict, Optional

import numpy as np
import torch

from .config import ModelConfig, RenderConfig
from .metrics import LPIPSMetric, compute_mse, compute_psnr, compute_ssim
from .model import NeRF
from .noise import NoiseConfig, add_noise_to_pose, compute_pose_error, set_noise_seed
from .rendering import NeRFRenderer
from .train import render_image


def load_checkpoint(checkpoint_path: Path, device: str = "cuda") -> tuple:
    """Reference inference.py:33-72 -> (renderer, config dict, iteration).  Loads with
    ``weights_only=True``: a checkpoint is tensors, dicts, lists and scalars only."""
    ckpt = torch.load(checkpoint_path, map_location=device, weights_only=True)
    cfg = ckpt.get("config", {})
    model_cfg = ModelConfig(**cfg.get("model", {}))
    # MI355X-only knob, kept out of config["model"] so reference loaders accept the file
    model_cfg.precision = ckpt.get("mi355x", {}).get("precision", model_cfg.precision)
    render_cfg = RenderConfig(**cfg.get("render", {}))
    coarse = NeRF(model_cfg).to(device)
    coarse.load_state_dict(ckpt["model_coarse"])
    coarse.eval()
    fine = None
    if "model_fine" in ckpt:
        fine = NeRF(model_cfg).to(device)
        fine.load_state_dict(ckpt["model_fine"])
        fine.eval()
    return NeRFRenderer(coarse, fine, render_cfg), cfg, ckpt.get("iteration", 0)


def save_image(img: torch.Tensor, path: Path) -> None:
    """Reference inference.py:108-111: [0,1] float (H,W,3) -> 8-bit PNG."""
    from PIL import Image
    arr = (img.detach().cpu().numpy() * 255).clip(0, 255).astype(np.uint8)
    Image.fromarray(arr).save(path)


def depth_to_colormap(depth: torch.Tensor) -> torch.Tensor:
    """Reference inference.py:114-125: min-max normalised depth through a turbo-like ramp."""
    depth = depth.detach().cpu()
    n = (depth - depth.min()) / (depth.max() - depth.min() + 1e-8)
    return torch.stack([torch.clamp(4 * n - 1.5, 0, 1), torch.clamp(2 - 4 * torch.abs(n - 0.5), 0, 1),
                        torch.clamp(1.5 - 4 * n, 0, 1)], dim=-1)


def generate_output_folder_name(mode: str, noise_config: NoiseConfig, scene: str) -> str:
    """Reference inference.py:128-142: ``{mode}_{scene}_{noise}_{timestamp}``."""
    return f"{mode}_{scene}_{noise_config}_{datetime.now().strftime('%Y%m%d_%H%M%S')}"


def create_spiral_poses(n_frames: int = 120, radius: float = 0.5, height: float = 0.0, n_rotations: float = 2.0,
                        device: str = "cuda") -> torch.Tensor:
    """Reference inference.py:321-362: look-at-origin cameras on a circle of radius 4."""
    t = np.arange(n_frames) / n_frames
    theta = 2 * np.pi * n_rotations * t
    pos = np.stack([4.0 * np.cos(theta), 4.0 * np.sin(theta), np.full_like(theta, height)], -1)
    fwd = -pos / np.linalg.norm(pos, axis=-1, keepdims=True)
    right = np.cross(fwd, np.array([0.0, 0.0, 1.0]))
    right /= np.linalg.norm(right, axis=-1, keepdims=True)
    up = np.cross(right, fwd)
    c2w = np.tile(np.eye(4, dtype=np.float32), (n_frames, 1, 1))
    c2w[:, :3, 0], c2w[:, :3, 1], c2w[:, :3, 2], c2w[:, :3, 3] = right, up, -fwd, pos
    return torch.from_numpy(c2w).to(device)


def _noisy_poses(test_data, noise_config: NoiseConfig):
    """Every view's (pose, noise info) in view order, as the reference's loop draws them."""
    if noise_config.seed is not None:
        set_noise_seed(noise_config.seed)
    out = []
    for i in range(test_data.images.shape[0]):
        orig = test_data.poses[i]
        if noise_config.has_noise:
            pose, info = add_noise_to_pose(orig, rotation_noise_deg=noise_config.rotation_noise_deg,
                                           translation_noise=noise_config.translation_noise)
            info.update(compute_pose_error(orig, pose))
        else:
            pose, info = orig, {}
        out.append((pose, info))
    return out


@torch.no_grad()
def evaluate_test_set(renderer: NeRFRenderer, test_data, output_dir: Path, noise_config: NoiseConfig,
                      device: str = "cuda", chunk_size: int = 1024 * 4, process_group=None,
                      save_images: bool = True, log=print) -> Dict[str, object]:
    """Reference inference.py:145-318 (same per-image records, summary keys and files),
    sharded over ``process_group``'s ranks when one is given."""
    rank, world = 0, 1
    if process_group is not None:
        import torch.distributed as dist
        rank, world = dist.get_rank(process_group), dist.get_world_size(process_group)
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    views = _noisy_poses(test_data, noise_config)
    if world > 1 and noise_config.has_noise and noise_config.seed is None:
        # unseeded noise: every rank must still render rank 0's draws
        obj = [[(p.cpu(), info) for p, info in views]]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(process_group, 0), group=process_group)
        views = [(p.to(test_data.poses.device), info) for p, info in obj[0]]
    lpips_metric = LPIPSMetric(device=device)
    n_images = test_data.images.shape[0]
    if rank == 0:
        log(f"Evaluating {n_images} test images on {world} rank(s)...")
    mine = []
    for i in range(rank, n_images, world):
        pose, noise_info = views[i]
        target = test_data.images[i]
        start = time.time()
        out = render_image(renderer, pose, test_data.H, test_data.W, test_data.focal, chunk_size=chunk_size)
        pred = out["rgb"]
        torch.cuda.synchronize() if pred.is_cuda else None
        rec = {"image": i, "psnr": compute_psnr(pred, target).item(), "ssim": compute_ssim(pred, target).item(),
               "mse": compute_mse(pred, target).item(), "render_time": time.time() - start}
        if noise_info:
            rec.update({f"noise_{k}": v for k, v in noise_info.items()})
        lp = lpips_metric(pred, target) if lpips_metric.available else None
        if lp is not None:
            rec["lpips"] = lp.item()
        mine.append(rec)
        if save_images:
            save_image(pred, output_dir / f"pred_{i:03d}.png")
            save_image(target, output_dir / f"gt_{i:03d}.png")
            save_image(torch.cat([target, pred], dim=1), output_dir / f"comparison_{i:03d}.png")
            save_image(depth_to_colormap(out["depth"]), output_dir / f"depth_{i:03d}.png")
        log(f"  Image {i + 1}/{n_images}: PSNR={rec['psnr']:.2f}, SSIM={rec['ssim']:.4f}, "
            f"time={rec['render_time']:.2f}s")
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine, group=process_group)
        per_image = sorted((r for part in gathered for r in part), key=lambda r: r["image"])
    else:
        per_image = mine
    psnr = [r["psnr"] for r in per_image]
    ssim = [r["ssim"] for r in per_image]
    mse = [r["mse"] for r in per_image]
    avg = {"psnr_mean": float(np.mean(psnr)), "psnr_std": float(np.std(psnr)), "ssim_mean": float(np.mean(ssim)),
           "ssim_std": float(np.std(ssim)), "mse_mean": float(np.mean(mse)), "mse_std": float(np.std(mse)),
           "n_images": n_images}
    lp = [r["lpips"] for r in per_image if "lpips" in r]
    if lp:
        avg["lpips_mean"], avg["lpips_std"] = float(np.mean(lp)), float(np.std(lp))
    if noise_config.has_noise:
        rot = [r.get("noise_rotation_error_deg", 0) for r in per_image]
        tr = [r.get("noise_translation_error", 0) for r in per_image]
        avg["noise_config"] = {"rotation_noise_deg": noise_config.rotation_noise_deg,
                               "translation_noise": noise_config.translation_noise, "seed": noise_config.seed}
        avg["actual_noise"] = {"rotation_error_mean_deg": float(np.mean(rot)),
                               "rotation_error_std_deg": float(np.std(rot)),
                               "translation_error_mean": float(np.mean(tr)),
                               "translation_error_std": float(np.std(tr))}
    if rank == 0:
        (output_dir / "per_image_metrics.json").write_text(json.dumps(per_image, indent=2))
        (output_dir / "test_metrics.json").write_text(json.dumps(avg, indent=2))
        (output_dir / "experiment_config.json").write_text(json.dumps({
            "mode": "test",
            "noise_config": {"rotation_noise_deg": noise_config.rotation_noise_deg,
                             "translation_noise": noise_config.translation_noise, "seed": noise_config.seed},
            "timestamp": datetime.now().isoformat(), "output_dir": str(output_dir), "ranks": world}, indent=2))
    return avg


__all__ = ["load_checkpoint", "render_image", "save_image", "depth_to_colormap", "generate_output_folder_name",
           "create_spiral_poses", "evaluate_test_set"]
