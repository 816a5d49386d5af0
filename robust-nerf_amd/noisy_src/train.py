"""
NeRF training entry point — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src/train.py``.

* ``train_step(renderer, optimizer, batch)`` keeps the reference's signature and
  returned metrics (train.py:68-119: host syncs for the logged scalars, joint clip at
  1.0 over both networks).  With the package's ``FusedAdam`` the clip folds into the
  fused update.
* ``train(config, noise_config)`` is the reference loop (train.py:307-577): seed,
  data (optionally with fixed pose noise), both networks, Adam + LambdaLR, one CSV
  row per iteration, validation + checkpoint every ``val_every`` (``checkpoint_best``
  on a new best PSNR), a plain checkpoint every ``save_every``, a final checkpoint,
  the final evaluation on every validation view and ``summary.json``.  The step
  itself is ``engine.Trainer`` (HIP kernels, no host syncs); the logged scalars are
  read once per iteration as the reference does.
* Data parallel (``torchrun --nproc-per-node N -m noisy_src.train ...``): every rank
  draws the SAME global batch and random numbers (identical seeds), takes its
  contiguous slice, and the gradients are averaged over RCCL inside
  the backward; ``--batch_size`` stays the global batch.  Rank 0 logs, validates and
  writes the checkpoints.
* ``save_checkpoint`` / ``load_checkpoint`` keep the reference's format; the MI355X
  precision knob is stored under a separate top-level key so the reference's
  ``ModelConfig(**cfg["model"])`` still loads the file.
"""

from __future__ import annotations

import json
import math
import random
import time
from datetime import datetime
from pathlib import Path
from typing import Dict, Optional

import numpy as np
import torch

from . import ops
from .config import NeRFConfig
from .data import BlenderData, RayDataset, RaySampler, create_data_loaders
from .engine import GraphedTrainer, LaggedScalars, Trainer, check_run_args, init_distributed, mean_over_ranks, rank_slice
from .logger import ExperimentLogger, TrainingMetrics, ValidationMetrics
from .metrics import LPIPSMetric, compute_mse, compute_psnr, compute_ssim
from .model import create_nerf
from .noise import NoiseConfig
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


def generate_experiment_name(scene: str, noise_config: Optional[NoiseConfig], base_name: str = "") -> str:
    """Reference train.py:44-66: ``{scene}[_{base}]_{noise|clean}_{timestamp}``."""
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    noise_desc = str(noise_config) if noise_config is not None and noise_config.has_noise else "clean"
    return f"{scene}_{base_name}_{noise_desc}_{ts}" if base_name else f"{scene}_{noise_desc}_{ts}"


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
    rays_o, rays_d = get_rays(dirs, pose.detach().contiguous())
    out = renderer(rays_o.reshape(-1, 3), rays_d.reshape(-1, 3), chunk_size=chunk_size, is_train=False)
    key = "fine" if "rgb_fine" in out else "coarse"
    return {"rgb": out[f"rgb_{key}"].reshape(H, W, 3), "depth": out[f"depth_{key}"].reshape(H, W),
            "acc": out[f"acc_{key}"].reshape(H, W)}


@torch.no_grad()
def evaluate(renderer: NeRFRenderer, val_data: BlenderData, logger: Optional[ExperimentLogger] = None,
             iteration: int = 0, num_images: int = 5, lpips_metric: Optional[LPIPSMetric] = None,
             chunk_size: int = 1024 * 4) -> ValidationMetrics:
    """Reference train.py:163-233: mean PSNR / SSIM / MSE (+ LPIPS when available) over
    the first ``num_images`` validation views; PNGs of the first three when a logger is
    given."""
    psnr, ssim, mse, lp = [], [], [], []
    for i in range(min(num_images, val_data.images.shape[0])):
        out = render_image(renderer, val_data.poses[i], val_data.H, val_data.W, val_data.focal, chunk_size)
        pred, target = out["rgb"], val_data.images[i]
        mse.append(compute_mse(pred, target).item())
        psnr.append(compute_psnr(pred, target).item())
        ssim.append(compute_ssim(pred, target).item())
        if lpips_metric is not None:
            v = lpips_metric(pred, target)
            if v is not None:
                lp.append(v.item())
        if logger is not None and i < 3:
            logger.log_images(f"val_{i}", pred, target, iteration, depth=out["depth"])
    return ValidationMetrics(iteration=iteration, psnr=float(np.mean(psnr)), ssim=float(np.mean(ssim)),
                             mse=float(np.mean(mse)), lpips=float(np.mean(lp)) if lp else None,
                             per_image_psnr=psnr, per_image_ssim=ssim)


def _plain(d: dict) -> dict:
    """Config values made plain (Path -> str, tuple -> list) so that the file reads back
    with ``torch.load(..., weights_only=True)``."""
    return {k: str(v) if isinstance(v, Path) else list(v) if isinstance(v, tuple) else v for k, v in d.items()}


def checkpoint_config(config: NeRFConfig) -> dict:
    """The reference's ``checkpoint["config"]`` (train.py:256-264).  ``ModelConfig.precision``
    (an MI355X-only field) is left out so the reference's ``ModelConfig(**cfg["model"])``
    accepts it; it travels under ``checkpoint["mi355x"]``."""
    model = {k: v for k, v in config.model.__dict__.items() if k != "precision"}
    return {"model": _plain(model), "render": _plain(config.render.__dict__), "data": _plain(config.data.__dict__),
            "train": _plain(config.train.__dict__)}


def noise_dict(noise_config: NoiseConfig) -> dict:
    return {"rotation_noise_deg": noise_config.rotation_noise_deg, "translation_noise": noise_config.translation_noise,
            "translation_noise_pct": noise_config.translation_noise_pct, "seed": noise_config.seed}


def save_checkpoint(output_dir, iteration: int, model_coarse, model_fine, optimizer: torch.optim.Optimizer,
                    config: NeRFConfig, noise_config=None, metrics: Optional[Dict] = None,
                    is_best: bool = False) -> None:
    """Reference train.py:236-286: same keys (iteration, model_coarse/_fine state_dicts in
    nn.Linear naming, optimizer state, config as plain dicts), same file names."""
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    ckpt = {"iteration": iteration, "model_coarse": model_coarse.state_dict(), "optimizer": optimizer.state_dict(),
            "config": checkpoint_config(config), "mi355x": {"precision": getattr(config.model, "precision", "fp32")}}
    if model_fine is not None:
        ckpt["model_fine"] = model_fine.state_dict()
    if metrics is not None:
        ckpt["metrics"] = metrics
    if noise_config is not None:
        ckpt["noise_config"] = noise_dict(noise_config)
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


def train(config: NeRFConfig, noise_config: Optional[NoiseConfig] = None, *,
          train_data: Optional[BlenderData] = None, val_data: Optional[BlenderData] = None,
          process_group=None, log=print, graph: bool = False) -> Dict[str, object]:
    """Reference train.py:307-577.  ``train_data`` / ``val_data`` (optional) replace the
    on-disk scene; ``process_group`` (or a torchrun environment, see ``main``) makes it
    data parallel.  ``graph`` replays the training step from a hipGraph after the first
    iteration (``engine.GraphedTrainer``; same results as eager); with data parallelism
    the RCCL all-reduces are captured into it too (``nccl`` backend only).
    Returns the networks, the output directory and the final metrics."""
    import torch.distributed as dist

    rank, world = 0, 1
    if process_group is not None:
        rank, world = dist.get_rank(process_group), dist.get_world_size(process_group)
    check_run_args(config, world, train_data, val_data)
    if graph and world > 1 and dist.get_backend(process_group) != "nccl":
        # the captured step contains the all-reduce: only RCCL collectives are graph-capturable
        raise ValueError("train(graph=True) with data parallelism needs the nccl (RCCL) backend")
    set_seed(config.train.seed)
    device = config.train.device
    if device.startswith("cuda") and not torch.cuda.is_available():
        raise RuntimeError("noisy_src.train needs a ROCm device (the reference falls back to its CPU path; "
                           "this framework has no CPU path)")
    exp_name = config.train.experiment_name
    if exp_name in ("auto", ""):
        exp_name = generate_experiment_name(config.data.scene_name, noise_config)
    output_dir = Path(config.train.output_dir) / exp_name
    logger = ExperimentLogger(output_dir, exp_name, use_tensorboard=True) if rank == 0 else None
    if logger is not None:
        logger.log_config(config)

    if train_data is None:
        sampler, train_data, val_data = create_data_loaders(config.data, device=device, noise_config=noise_config)
    else:
        sampler = RaySampler(RayDataset(train_data, config.data.batch_size, noise_config=noise_config),
                             config.data.batch_size, shuffle=config.data.shuffle)
    model_coarse, model_fine = create_nerf(config.model)
    model_coarse = model_coarse.to(device)
    model_fine = model_fine.to(device) if config.render.use_hierarchical else None
    if logger is not None:
        logger.log_model_info(model_coarse, "model_coarse")
        if model_fine is not None:
            logger.log_model_info(model_fine, "model_fine")
    renderer = NeRFRenderer(model_coarse, model_fine, config.render)
    # coarse_stream="auto": the coarse chain becomes a second graph branch only in a
    # --graph replay of <= 1024 rays (engine.Trainer), where it pays
    trainer = Trainer(model_coarse, model_fine, config.render, lr=config.train.lr, lr_decay=config.train.lr_decay,
                      process_group=process_group, coarse_stream="auto")
    optimizer = trainer.optimizer
    lpips_metric = LPIPSMetric(device=device) if rank == 0 else None
    if lpips_metric is not None and not lpips_metric.available:
        lpips_metric = None
    if rank == 0:
        nc = noise_config
        (output_dir / "experiment_config.json").write_text(json.dumps({
            "scene": config.data.scene_name, "experiment_name": exp_name,
            "noise_config": {"rotation_noise_deg": nc.rotation_noise_deg if nc else 0,
                             "translation_noise": nc.translation_noise if nc else 0,
                             "translation_noise_pct": nc.translation_noise_pct if nc else 0,
                             "seed": nc.seed if nc else None, "has_noise": nc.has_noise if nc else False},
            "num_iterations": config.train.num_iterations, "batch_size": config.data.batch_size,
            "img_scale": config.data.img_scale, "timestamp": datetime.now().isoformat(),
            "data_parallel_ranks": world}, indent=2))
        log(f"NeRF training: {exp_name} -> {output_dir} ({world} rank(s), {sampler.n_rays:,} rays, "
            f"{train_data.H}x{train_data.W}, focal {train_data.focal:.2f})")

    B = config.data.batch_size
    rc = config.render
    start = time.time()
    best_psnr = 0.0
    iteration = 0
    graphed = None
    lagged = LaggedScalars()  # logged losses read one iteration late: no per-step host sync
    t_prev = time.time()

    def log_iteration(done):
        if done is None or logger is None:
            return
        vals, (it, keys, lr, batch_time) = done
        vm = dict(zip(keys, vals))
        last = vm.get("loss_fine", vm["loss_coarse"])
        psnr = -10.0 * math.log10(last) if last > 0 else float("inf")
        logger.log_training(TrainingMetrics(iteration=it, loss=vm["loss"], loss_coarse=vm["loss_coarse"],
                                            loss_fine=vm.get("loss_fine"), psnr=psnr, learning_rate=lr,
                                            time_per_iter=batch_time, rays_per_sec=B / batch_time))
        if it % config.train.log_every == 0:
            log(f"[{it:7d}/{config.train.num_iterations}] loss: {vm['loss']:.5f} | psnr: {psnr:.2f} | "
                f"lr: {lr:.2e} | rays/s: {B / batch_time:.0f} | time: {(time.time() - start) / 60:.1f}min")

    while iteration < config.train.num_iterations:
        for batch in sampler:
            if iteration >= config.train.num_iterations:
                break
            n = batch["rays_o"].shape[0]
            if world > 1 and n % world:
                # only an epoch's short final batch (batch_size % world == 0 is checked
                # up front): it cannot be split evenly over the ranks, so it is skipped
                continue
            # the global random draws, in the reference's order (jitter, then inverse-CDF
            # uniforms: rendering.py:161 -> rays.py:204, :255), identical on every rank
            t_rand = torch.rand(n, rc.num_samples, device=device) if rc.perturb else None
            u = torch.rand(n, rc.num_samples_fine, device=device) if (rc.use_hierarchical and model_fine) else None
            sl = rank_slice(n, rank, world) if world > 1 else slice(0, n)
            args = (batch["rays_o"][sl], batch["rays_d"][sl], batch["target_rgb"][sl],
                    None if t_rand is None else t_rand[sl], None if u is None else u[sl])
            if graph and graphed is None and iteration >= 1 and n == B:
                # captured after one eager step (state exists), on a full batch: an epoch's
                # short tail batch would leave every full batch after it eager
                graphed = GraphedTrainer(trainer, *args, warmup=0)
            if graphed is not None and args[0].shape == graphed.static[0].shape:
                m = graphed.step(*args)
            else:  # eager (also an epoch's short final batch in graph mode)
                m = trainer.step(*args)
            keys = ["loss", "loss_coarse"] + (["loss_fine"] if "loss_fine" in m else [])
            now = time.time()
            log_iteration(lagged.push(mean_over_ranks([m[k] for k in keys], process_group),
                                      (iteration, keys, optimizer.param_groups[0]["lr"], now - t_prev)))
            t_prev = now
            if logger is not None and iteration > 0 and (iteration % config.train.val_every == 0
                                                         or iteration % config.train.save_every == 0):
                log_iteration(lagged.flush())
                if iteration % config.train.val_every == 0:
                    vmx = evaluate(renderer, val_data, logger, iteration, num_images=5, lpips_metric=lpips_metric)
                    logger.log_validation(vmx)
                    is_best = vmx.psnr > best_psnr
                    best_psnr = max(best_psnr, vmx.psnr)
                    log(f"  validation @ {iteration}: PSNR {vmx.psnr:.2f} dB, SSIM {vmx.ssim:.4f}"
                        + (" (best)" if is_best else ""))
                    save_checkpoint(output_dir, iteration, model_coarse, model_fine, optimizer, config, noise_config,
                                    metrics={"psnr": vmx.psnr, "ssim": vmx.ssim}, is_best=is_best)
                else:
                    save_checkpoint(output_dir, iteration, model_coarse, model_fine, optimizer, config, noise_config)
                t_prev = time.time()  # the next iteration's time excludes the validation
            iteration += 1
    log_iteration(lagged.flush())
    result = {"model_coarse": model_coarse, "model_fine": model_fine, "output_dir": output_dir,
              "best_psnr": best_psnr}
    if logger is not None:
        save_checkpoint(output_dir, iteration, model_coarse, model_fine, optimizer, config, noise_config)
        final = evaluate(renderer, val_data, logger, iteration, num_images=val_data.images.shape[0],
                         lpips_metric=lpips_metric)
        logger.log_validation(final)
        logger.save_summary()
        logger.close()
        log(f"final: PSNR {final.psnr:.2f} dB, SSIM {final.ssim:.4f}; {(time.time() - start) / 60:.1f} min; "
            f"results in {output_dir}")
        result["val"] = final
    if process_group is not None:
        dist.barrier(process_group)
    return result


def build_arg_parser():
    """Reference train.py:580-657 flags (same names and defaults) plus ``--precision`` and ``--graph``."""
    import argparse
    ap = argparse.ArgumentParser(description="Train NeRF with optional pose noise (MI355X HIP path)")
    ap.add_argument("--scene", type=str, default="lego")
    ap.add_argument("--data_root", type=str, default=None)
    ap.add_argument("--img_scale", type=float, default=0.5)
    ap.add_argument("--batch_size", type=int, default=1024, help="global batch (rays) over all ranks")
    ap.add_argument("--num_iters", type=int, default=200000)
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--no_hierarchical", action="store_true")
    ap.add_argument("--num_samples", type=int, default=64)
    ap.add_argument("--num_samples_fine", type=int, default=128)
    ap.add_argument("--rotation_noise", type=float, default=0.0)
    ap.add_argument("--translation_noise", type=float, default=0.0)
    ap.add_argument("--translation_noise_pct", type=float, default=0.0)
    ap.add_argument("--noise_seed", type=int, default=None)
    ap.add_argument("--log_every", type=int, default=100)
    ap.add_argument("--val_every", type=int, default=5000)
    ap.add_argument("--save_every", type=int, default=10000)
    ap.add_argument("--output_dir", type=str, default="outputs")
    ap.add_argument("--exp_name", type=str, default="auto")
    ap.add_argument("--device", type=str, default="cuda")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--precision", type=str, default="fp32", choices=["fp32", "bf16", "fp16"],
                    help="MLP operand precision (fp32 = the reference's numerics)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the training step from a hipGraph (same results as eager; with RCCL data "
                         "parallelism the all-reduces are captured too)")
    return ap


def main(argv=None) -> None:
    """``python -m noisy_src.train`` (or under ``torchrun`` for data parallelism)."""
    from .config import DataConfig, ModelConfig, RenderConfig, TrainConfig

    a = build_arg_parser().parse_args(argv)
    noise_config = None
    if a.rotation_noise > 0 or a.translation_noise > 0 or a.translation_noise_pct > 0:
        noise_config = NoiseConfig(rotation_noise_deg=a.rotation_noise, translation_noise=a.translation_noise,
                                   translation_noise_pct=a.translation_noise_pct, seed=a.noise_seed)
    pg, rank, world, device = init_distributed(a.device)
    cfg = NeRFConfig(
        model=ModelConfig(precision=a.precision),
        render=RenderConfig(use_hierarchical=not a.no_hierarchical, num_samples=a.num_samples,
                            num_samples_fine=a.num_samples_fine),
        data=DataConfig(scene_name=a.scene, data_root=Path(a.data_root) if a.data_root else None,
                        img_scale=a.img_scale, batch_size=a.batch_size),
        train=TrainConfig(lr=a.lr, num_iterations=a.num_iters, output_dir=Path(a.output_dir),
                          experiment_name=a.exp_name, device=device, seed=a.seed, log_every=a.log_every,
                          val_every=a.val_every, save_every=a.save_every))
    if world > 1 and cfg.train.experiment_name in ("auto", ""):
        # one shared directory name for all ranks (rank 0's timestamp)
        import torch.distributed as dist
        name = [generate_experiment_name(a.scene, noise_config)]
        dist.broadcast_object_list(name, src=0, group=pg)
        cfg.train.experiment_name = name[0]
    train(cfg, noise_config, process_group=pg, graph=a.graph)
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


__all__ = ["set_seed", "generate_experiment_name", "train_step", "render_image", "evaluate", "save_checkpoint",
           "load_checkpoint", "train", "main"]

if __name__ == "__main__":
    main()
