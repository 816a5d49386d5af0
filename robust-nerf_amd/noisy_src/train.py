"""
NeRF training step and image rendering — drop-in for ShawnnnLiu/Robust-NeRF
``noisy_src/train.py`` (the functions on and around the hot path).

``train_step(renderer, optimizer, batch)`` keeps the reference's signature and
returned metrics (train.py:68-119: four host syncs for the logged scalars, joint
clip at 1.0 over both networks).  With the package's ``FusedAdam`` the clip folds
into the fused update.  ``engine.Trainer`` is the same step without the host syncs,
which is what ``bench.py`` times.  ``train`` is a minimal loop over a ``RaySampler``;
``save_checkpoint`` / ``load_checkpoint`` keep the reference's checkpoint format.
"""

from __future__ import annotations

import random
import time
from typing import Dict, Optional

import numpy as np
import torch

from . import ops
from .config import NeRFConfig
from .data import BlenderData, RayDataset, RaySampler
from .engine import Trainer, lr_lambda_factory
from .metrics import compute_mse, compute_psnr, compute_ssim
from .model import create_nerf
from .optim import FusedAdam, clip_grad_norm_
from .rays import get_ray_directions, get_rays
from .rendering import NeRFRenderer


def set_seed(seed: int) -> None:
    """Reference train.py:36-42."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def train_step(renderer: NeRFRenderer, optimizer: torch.optim.Optimizer, batch: Dict[str, torch.Tensor],
               t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None) -> Dict[str, float]:
    """Reference train.py:68-119 (``t_rand``/``u`` optionally inject the random draws)."""
    from .rendering import render_rays

    optimizer.zero_grad()
    out = render_rays(renderer.model_coarse, renderer.model_fine, batch["rays_o"], batch["rays_d"], renderer.config,
                      is_train=True, t_rand=t_rand, u=u)
    target = batch["target_rgb"]
    loss_c = ops.mse_loss(out["rgb_coarse"], target)
    metrics = {"loss_coarse": loss_c.item(), "psnr_coarse": compute_psnr(out["rgb_coarse"].detach(), target).item()}
    if "rgb_fine" in out:
        loss_f = ops.mse_loss(out["rgb_fine"], target)
        loss = loss_c + loss_f
        metrics["loss_fine"] = loss_f.item()
        metrics["psnr_fine"] = compute_psnr(out["rgb_fine"].detach(), target).item()
        metrics["psnr"] = metrics["psnr_fine"]
    else:
        loss = loss_c
        metrics["loss_fine"] = None
        metrics["psnr"] = metrics["psnr_coarse"]
    metrics["loss"] = loss.item()
    loss.backward()
    params = list(renderer.parameters())
    if isinstance(optimizer, FusedAdam):
        optimizer.step(clip_groups=[(params, 1.0)])
    else:
        clip_grad_norm_(params, 1.0)
        optimizer.step()
    return metrics


@torch.no_grad()
def render_image(renderer: NeRFRenderer, pose: torch.Tensor, H: int, W: int, focal: float,
                 chunk_size: int = 1024 * 4) -> Dict[str, torch.Tensor]:
    """Reference train.py:122-160: every pixel of one view, deterministic (is_train=False)."""
    dirs = get_ray_directions(H, W, focal, device=pose.device)
    rays_o, rays_d = get_rays(dirs, pose.contiguous())
    out = renderer(rays_o.reshape(-1, 3), rays_d.reshape(-1, 3), chunk_size=chunk_size, is_train=False)
    key = "fine" if "rgb_fine" in out else "coarse"
    return {"rgb": out[f"rgb_{key}"].reshape(H, W, 3), "depth": out[f"depth_{key}"].reshape(H, W),
            "acc": out[f"acc_{key}"].reshape(H, W)}


@torch.no_grad()
def evaluate(renderer: NeRFRenderer, val_data: BlenderData, num_images: int = 5,
             chunk_size: int = 1024 * 4) -> Dict[str, object]:
    """Reference train.py:164-233 without the logger: mean PSNR / SSIM / MSE over the
    first ``num_images`` validation views."""
    psnr, ssim, mse = [], [], []
    for i in range(min(num_images, val_data.images.shape[0])):
        out = render_image(renderer, val_data.poses[i], val_data.H, val_data.W, val_data.focal, chunk_size)
        pred, target = out["rgb"], val_data.images[i]
        mse.append(compute_mse(pred, target).item())
        psnr.append(compute_psnr(pred, target).item())
        ssim.append(compute_ssim(pred, target).item())
    return {"psnr": float(np.mean(psnr)), "ssim": float(np.mean(ssim)), "mse": float(np.mean(mse)),
            "per_image_psnr": psnr, "per_image_ssim": ssim}


def save_checkpoint(output_dir, iteration: int, model_coarse, model_fine, optimizer: torch.optim.Optimizer,
                    config: NeRFConfig, noise_config=None, metrics: Optional[Dict] = None,
                    is_best: bool = False) -> None:
    """Reference train.py:236-286: same keys (iteration, model_coarse/_fine state_dicts in
    nn.Linear naming, optimizer state, config as plain dicts), same file names.  The config
    values are made plain (Path -> str, tuple -> list) so that ``torch.load(...,
    weights_only=True)`` reads the file back."""
    from pathlib import Path

    def plain(d):
        return {k: str(v) if isinstance(v, Path) else list(v) if isinstance(v, tuple) else v for k, v in d.items()}

    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    ckpt = {"iteration": iteration, "model_coarse": model_coarse.state_dict(), "optimizer": optimizer.state_dict(),
            "config": {"model": plain(config.model.__dict__), "render": plain(config.render.__dict__),
                       "data": plain(config.data.__dict__), "train": plain(config.train.__dict__)}}
    if model_fine is not None:
        ckpt["model_fine"] = model_fine.state_dict()
    if metrics is not None:
        ckpt["metrics"] = metrics
    if noise_config is not None:
        ckpt["noise_config"] = {"rotation_noise_deg": noise_config.rotation_noise_deg,
                                "translation_noise": noise_config.translation_noise,
                                "translation_noise_pct": noise_config.translation_noise_pct,
                                "seed": noise_config.seed}
    torch.save(ckpt, output_dir / f"checkpoint_{iteration:07d}.pt")
    torch.save(ckpt, output_dir / "checkpoint_latest.pt")
    if is_best:
        torch.save(ckpt, output_dir / "checkpoint_best.pt")


def load_checkpoint(checkpoint_path, model_coarse, model_fine, optimizer: Optional[torch.optim.Optimizer] = None) -> int:
    """Reference train.py:289-304 -> iteration (``weights_only=True``)."""
    ckpt = torch.load(checkpoint_path, map_location=next(model_coarse.parameters()).device, weights_only=True)
    model_coarse.load_state_dict(ckpt["model_coarse"])
    if model_fine is not None and "model_fine" in ckpt:
        model_fine.load_state_dict(ckpt["model_fine"])
    if optimizer is not None and "optimizer" in ckpt:
        optimizer.load_state_dict(ckpt["optimizer"])
    return ckpt.get("iteration", 0)


def train(config: NeRFConfig, train_data: BlenderData, val_data: Optional[BlenderData] = None,
          num_iterations: Optional[int] = None, log=print) -> Dict[str, object]:
    """Reference train.py:307-577, minus logging/checkpoint I/O: seeds, builds the two
    networks and the fused Adam + LambdaLR, iterates the epoch sampler, steps."""
    set_seed(config.train.seed)
    coarse, fine = create_nerf(config.model)
    dev = train_data.images.device
    coarse, fine = coarse.to(dev), fine.to(dev) if fine is not None else None
    trainer = Trainer(coarse, fine, config.render, lr=config.train.lr, lr_decay=config.train.lr_decay)
    sampler = RaySampler(RayDataset(train_data, batch_size=config.data.batch_size), config.data.batch_size,
                         shuffle=config.data.shuffle)
    it = iter(sampler)
    n_iter = num_iterations if num_iterations is not None else config.train.num_iterations
    t0 = time.time()
    history = []
    for step in range(n_iter):
        try:
            batch = next(it)
        except StopIteration:
            it = iter(sampler)
            batch = next(it)
        m = trainer.step(batch["rays_o"], batch["rays_d"], batch["target_rgb"])
        if (step + 1) % config.train.log_every == 0 or step == n_iter - 1:
            loss = float(m["loss"])
            history.append((step, loss))
            log(f"iter {step + 1}: loss {loss:.5f} lr {trainer.scheduler.get_last_lr()[0]:.4e} "
                f"({(time.time() - t0) / (step + 1) * 1e3:.2f} ms/it)")
    result = {"model_coarse": coarse, "model_fine": fine, "history": history}
    if val_data is not None:
        result["val"] = evaluate(NeRFRenderer(coarse, fine, config.render), val_data)
    return result


def main(argv=None) -> None:
    """``python -m noisy_src.train`` — the reference CLI (train.py:580-640), same flags
    plus ``--precision``; needs the NeRF synthetic scene under ``--data_root``."""
    import argparse
    from pathlib import Path

    from .config import DataConfig, ModelConfig, RenderConfig, TrainConfig
    from .data import load_blender_data
    from .logger import ExperimentLogger, ValidationMetrics

    ap = argparse.ArgumentParser(description="NeRF training (MI355X HIP path)")
    ap.add_argument("--scene", type=str, default="lego")
    ap.add_argument("--data_root", type=str, default=None)
    ap.add_argument("--img_scale", type=float, default=0.5)
    ap.add_argument("--batch_size", type=int, default=1024)
    ap.add_argument("--num_iters", type=int, default=200000)
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--no_hierarchical", action="store_true")
    ap.add_argument("--num_samples", type=int, default=64)
    ap.add_argument("--num_samples_fine", type=int, default=128)
    ap.add_argument("--log_every", type=int, default=100)
    ap.add_argument("--val_every", type=int, default=5000)
    ap.add_argument("--output_dir", type=str, default="outputs")
    ap.add_argument("--exp_name", type=str, default="auto")
    ap.add_argument("--device", type=str, default="cuda")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--precision", type=str, default="fp32", choices=["fp32", "bf16", "fp16"])
    a = ap.parse_args(argv)
    cfg = NeRFConfig(
        model=ModelConfig(precision=a.precision),
        render=RenderConfig(num_samples=a.num_samples, num_samples_fine=a.num_samples_fine,
                            use_hierarchical=not a.no_hierarchical),
        data=DataConfig(scene_name=a.scene, data_root=Path(a.data_root) if a.data_root else None,
                        img_scale=a.img_scale, batch_size=a.batch_size),
        train=TrainConfig(lr=a.lr, num_iterations=a.num_iters, log_every=a.log_every, val_every=a.val_every,
                          output_dir=Path(a.output_dir), experiment_name=a.exp_name, device=a.device, seed=a.seed))
    root = cfg.data.data_root or Path("data") / "raw"
    train_data = load_blender_data(root, a.scene, "train", a.img_scale, a.device)
    val_data = load_blender_data(root, a.scene, "val", a.img_scale, a.device)
    name = a.exp_name if a.exp_name != "auto" else f"{a.scene}_clean_{time.strftime('%Y%m%d_%H%M%S')}"
    logger = ExperimentLogger(Path(a.output_dir) / name, name)
    logger.log_config(cfg)
    res = train(cfg, train_data, val_data)
    if "val" in res:
        v = res["val"]
        logger.log_validation(ValidationMetrics(iteration=a.num_iters, psnr=v["psnr"], ssim=v["ssim"], mse=v["mse"],
                                                per_image_psnr=v["per_image_psnr"], per_image_ssim=v["per_image_ssim"]))
    logger.close()


__all__ = ["set_seed", "train_step", "render_image", "evaluate", "save_checkpoint", "load_checkpoint", "train",
           "lr_lambda_factory", "main"]

if __name__ == "__main__":
    main()
