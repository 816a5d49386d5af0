"""
Joint NeRF + camera-pose training step — drop-in for ShawnnnLiu/Robust-NeRF
``noisy_src/train_pose_opt.py`` (the pieces on the hot path).

* ``CameraPoseParameters`` keeps the reference's parameterisation (axis-angle
  rotation deltas and translation deltas, both (N,3), zero-initialised;
  ``R = R_delta(w) R_init``, ``t = t_init + dt``) and its ``theta < 1e-6 -> I``
  quirk that blocks dL/dw at w = 0 (train_pose_opt.py:143-161; Appendix A.1).
  ``get_poses`` is one HIP kernel (``nr_se3_poses_fwd``/``_bwd``).  The two deltas
  are views of one flat 16-B-aligned buffer, so the pose Adam is one fused launch.
* ``train_step_with_poses`` follows train_pose_opt.py:290-411 step for step: poses ->
  rays (one gather kernel) -> render -> MSE coarse+fine -> L2 pose regularisers ->
  backward -> separate clips (coarse 1.0, fine 1.0, poses 0.1) -> the two optimizers.
* ``train_with_pose_optimization(config, noise_config, init_mode, ...)`` is the
  reference loop (train_pose_opt.py:613-1054): noisy or clean initial poses, the pose
  Adam and its LambdaLR only after ``pose_opt_delay``, one CSV row per iteration,
  validation + pose errors + checkpoint every ``val_every``, checkpoints every
  ``save_every``, the final evaluation and checkpoint, ``final_poses.pt`` and
  ``summary.json``.  The step is ``engine.PoseTrainer`` (HIP, no host syncs).  Under
  ``torchrun`` it is data parallel exactly like ``train.train``: identical global draws
  on every rank, contiguous slices, network and pose gradients averaged over RCCL.
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
import torch.nn as nn

from . import ops
from .config import RenderConfig
from .config import NeRFConfig
from .data import BlenderData, load_blender_data
from .data_pose_opt import PixelBatch, PixelSampler, create_pixel_dataset
from .engine import LaggedScalars, PoseTrainer, check_run_args, init_distributed, mean_over_ranks, rank_slice
from .logger import ExperimentLogger, TrainingMetrics, ValidationMetrics
from .metrics import LPIPSMetric, compute_mse, compute_psnr, compute_ssim
from .model import NeRF
from .noise import NoiseConfig, add_noise_to_poses, compute_pose_error
from .optim import FusedAdam, clip_grad_norm_
from .rays import get_ray_directions, get_rays
from .rendering import render_rays


def set_seed(seed: int) -> None:
    """Reference train_pose_opt.py:44-50."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


class CameraPoseParameters(nn.Module):
    """Reference train_pose_opt.py:53-271."""

    def __init__(self, initial_poses: torch.Tensor, learn_rotation: bool = True, learn_translation: bool = True,
                 fixed_small_angle: bool = False):
        super().__init__()
        self.n_poses = initial_poses.shape[0]
        self.learn_rotation = learn_rotation
        self.learn_translation = learn_translation
        # opt-in: exact Rodrigues derivative at w = 0 instead of the reference's blocked gradient
        self.fixed_small_angle = fixed_small_angle
        self.register_buffer("initial_poses", initial_poses.clone().float().contiguous())
        dev = initial_poses.device
        flat = torch.zeros(2 * self.n_poses * 3 + 4, device=dev)  # 16-B aligned halves
        off_t = ((self.n_poses * 3 + 3) // 4) * 4
        rot = flat[:self.n_poses * 3].view(self.n_poses, 3)
        trans = flat[off_t:off_t + self.n_poses * 3].view(self.n_poses, 3)
        if learn_rotation:
            self.rotation_deltas = nn.Parameter(rot)
        else:
            self.register_buffer("rotation_deltas", rot)
        if learn_translation:
            self.translation_deltas = nn.Parameter(trans)
        else:
            self.register_buffer("translation_deltas", trans)

    def _skew_symmetric(self, v: torch.Tensor) -> torch.Tensor:
        """Reference train_pose_opt.py:165-184."""
        z = torch.zeros(v.shape[0], device=v.device)
        return torch.stack([torch.stack([z, -v[:, 2], v[:, 1]], -1), torch.stack([v[:, 2], z, -v[:, 0]], -1),
                            torch.stack([-v[:, 1], v[:, 0], z], -1)], dim=1)

    def axis_angle_to_rotation_matrix(self, axis_angle: torch.Tensor) -> torch.Tensor:
        """Reference train_pose_opt.py:122-163, on the HIP SE(3) kernel (identity base pose)."""
        shape = axis_angle.shape[:-1]
        aa = axis_angle.reshape(-1, 3).float()
        eye = torch.eye(4, device=aa.device).expand(aa.shape[0], 4, 4).contiguous()
        R = ops.se3_poses(eye, aa, None, None, fixed_small_angle=self.fixed_small_angle)[:, :3, :3]
        return R.reshape(*shape, 3, 3)

    def get_poses(self, indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reference train_pose_opt.py:186-226 -> (N or len(indices), 4, 4)."""
        return ops.se3_poses(self.initial_poses, self.rotation_deltas if self.learn_rotation else None,
                             self.translation_deltas if self.learn_translation else None, indices,
                             fixed_small_angle=self.fixed_small_angle)

    def get_all_poses(self) -> torch.Tensor:
        return self.get_poses()

    def compute_pose_errors(self, ground_truth_poses: torch.Tensor,
                            indices: Optional[torch.Tensor] = None) -> Dict[str, float]:
        """Reference train_pose_opt.py:232-271."""
        with torch.no_grad():
            cur = self.get_poses(indices).cpu()
        gt = (ground_truth_poses[indices] if indices is not None else ground_truth_poses).cpu()
        errs = [compute_pose_error(gt[i], cur[i]) for i in range(cur.shape[0])]
        r = [e["rotation_error_deg"] for e in errs]
        t = [e["translation_error"] for e in errs]
        return {
            "rotation_error_mean": float(np.mean(r)), "rotation_error_std": float(np.std(r)),
            "rotation_error_max": float(np.max(r)), "translation_error_mean": float(np.mean(t)),
            "translation_error_std": float(np.std(t)), "translation_error_max": float(np.max(t)),
        }


def train_step_with_poses(model_coarse: NeRF, model_fine: Optional[NeRF], camera_params: CameraPoseParameters,
                          pixel_sampler: PixelSampler, optimizer_nerf: torch.optim.Optimizer,
                          optimizer_poses: Optional[torch.optim.Optimizer], pixel_batch: PixelBatch,
                          render_config: RenderConfig, optimize_poses: bool = True,
                          rotation_reg_weight: float = 0.0, translation_reg_weight: float = 0.0,
                          t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None) -> Dict[str, float]:
    """Reference train_pose_opt.py:290-411 (``t_rand``/``u`` optionally inject the draws)."""
    optimizer_nerf.zero_grad()
    if optimizer_poses is not None and optimize_poses:
        optimizer_poses.zero_grad()
    all_poses = camera_params.get_all_poses()
    rays_o, rays_d = pixel_sampler.get_rays_for_batch(pixel_batch, all_poses)
    target = pixel_batch.target_rgb
    out = render_rays(model_coarse, model_fine, rays_o, rays_d, render_config, is_train=True, t_rand=t_rand, u=u)
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
    if optimize_poses and (rotation_reg_weight > 0 or translation_reg_weight > 0):
        reg = 0.0
        if rotation_reg_weight > 0 and camera_params.learn_rotation:
            r = torch.mean(camera_params.rotation_deltas ** 2)
            reg = reg + rotation_reg_weight * r
            metrics["rotation_reg"] = r.item()
        if translation_reg_weight > 0 and camera_params.learn_translation:
            t = torch.mean(camera_params.translation_deltas ** 2)
            reg = reg + translation_reg_weight * t
            metrics["translation_reg"] = t.item()
        loss = loss + reg
        metrics["pose_reg_loss"] = reg.item() if isinstance(reg, torch.Tensor) else reg
    metrics["loss"] = loss.item()
    loss.backward()
    coarse = list(model_coarse.parameters())
    fine = list(model_fine.parameters()) if model_fine is not None else []
    poses = list(camera_params.parameters()) if (optimize_poses and optimizer_poses is not None) else []
    if isinstance(optimizer_nerf, FusedAdam):
        groups = [(coarse, 1.0)] + ([(fine, 1.0)] if fine else [])
        optimizer_nerf.step(clip_groups=groups)  # the clips fold into the fused update
    else:
        clip_grad_norm_(coarse, 1.0)
        if fine:
            clip_grad_norm_(fine, 1.0)
        optimizer_nerf.step()
    if optimizer_poses is not None and optimize_poses:
        if isinstance(optimizer_poses, FusedAdam):
            optimizer_poses.step(clip_groups=[(poses, 0.1)])
        else:
            clip_grad_norm_(poses, 0.1)
            optimizer_poses.step()
    return metrics


@torch.no_grad()
def render_image_with_pose(model_coarse: NeRF, model_fine: Optional[NeRF], pose: torch.Tensor, H: int, W: int,
                           focal: float, render_config: RenderConfig, chunk_size: int = 1024 * 4) -> Dict[str, torch.Tensor]:
    """Reference train_pose_opt.py:415-470."""
    dirs = get_ray_directions(H, W, focal, device=pose.device)
    rays_o, rays_d = get_rays(dirs, pose.contiguous())
    rays_o, rays_d = rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)
    key = "fine" if (model_fine is not None and render_config.use_hierarchical) else "coarse"
    rgb, depth, acc = [], [], []
    for i in range(0, rays_o.shape[0], chunk_size):
        o = render_rays(model_coarse, model_fine, rays_o[i:i + chunk_size], rays_d[i:i + chunk_size], render_config,
                        is_train=False)
        rgb.append(o[f"rgb_{key}"])
        depth.append(o[f"depth_{key}"])
        acc.append(o[f"acc_{key}"])
    return {"rgb": torch.cat(rgb).reshape(H, W, 3), "depth": torch.cat(depth).reshape(H, W),
            "acc": torch.cat(acc).reshape(H, W)}


@torch.no_grad()
def evaluate_with_poses(model_coarse: NeRF, model_fine: Optional[NeRF], camera_params: CameraPoseParameters,
                        val_data: BlenderData, val_indices: torch.Tensor, render_config: RenderConfig,
                        logger: Optional[ExperimentLogger] = None, iteration: int = 0, num_images: int = 5,
                        lpips_metric=None) -> ValidationMetrics:
    """Reference train_pose_opt.py:474-545: renders the first ``num_images`` validation
    views from their GROUND-TRUTH poses (the learnable poses are the training views');
    PNGs of the first three when a logger is given."""
    psnr, ssim, mse, lp = [], [], [], []
    for i, idx in enumerate(val_indices[:min(num_images, len(val_indices))]):
        idx = int(idx)
        out = render_image_with_pose(model_coarse, model_fine, val_data.poses[idx], val_data.H, val_data.W,
                                     val_data.focal, render_config)
        pred, target = out["rgb"], val_data.images[idx]
        mse.append(compute_mse(pred, target).item())
        psnr.append(compute_psnr(pred, target).item())
        ssim.append(compute_ssim(pred, target).item())
        if lpips_metric is not None:
            v = lpips_metric(pred, target)
            if v is not None:
                lp.append(v.item())
        if logger is not None and i < 3:
            logger.log_images(f"val_{idx}", pred, target, iteration, depth=out["depth"])
    return ValidationMetrics(iteration=iteration, psnr=float(np.mean(psnr)), ssim=float(np.mean(ssim)),
                             mse=float(np.mean(mse)), lpips=float(np.mean(lp)) if lp else None,
                             per_image_psnr=psnr, per_image_ssim=ssim)


def save_checkpoint_with_poses(output_dir, iteration: int, model_coarse, model_fine, camera_params,
                               optimizer_nerf, optimizer_poses, config: NeRFConfig, noise_config=None,
                               metrics: Optional[Dict] = None, pose_errors: Optional[Dict] = None,
                               is_best: bool = False) -> None:
    """Reference train_pose_opt.py:548-610: the train.py checkpoint plus ``camera_params``,
    ``optimizer_nerf`` / ``optimizer_poses``, ``initial_poses`` and ``pose_errors``."""
    from .train import checkpoint_config, noise_dict
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    ckpt = {"iteration": iteration, "model_coarse": model_coarse.state_dict(),
            "camera_params": camera_params.state_dict(), "optimizer_nerf": optimizer_nerf.state_dict(),
            "initial_poses": camera_params.initial_poses.cpu(), "config": checkpoint_config(config),
            "mi355x": {"precision": getattr(config.model, "precision", "fp32")}}
    if model_fine is not None:
        ckpt["model_fine"] = model_fine.state_dict()
    if optimizer_poses is not None:
        ckpt["optimizer_poses"] = optimizer_poses.state_dict()
    if metrics is not None:
        ckpt["metrics"] = metrics
    if pose_errors is not None:
        ckpt["pose_errors"] = pose_errors
    if noise_config is not None:
        ckpt["noise_config"] = noise_dict(noise_config)
    torch.save(ckpt, output_dir / f"checkpoint_{iteration:07d}.pt")
    torch.save(ckpt, output_dir / "checkpoint_latest.pt")
    if is_best:
        torch.save(ckpt, output_dir / "checkpoint_best.pt")


def generate_experiment_name(scene: str, noise_config: Optional[NoiseConfig], init_mode: str = "noisy") -> str:
    """Reference train_pose_opt.py:274-287."""
    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    noise_desc = str(noise_config) if noise_config is not None and noise_config.has_noise else "clean"
    return f"{scene}_poseopt_{init_mode}init_{noise_desc}_{ts}"


def train_with_pose_optimization(config: NeRFConfig, noise_config: Optional[NoiseConfig] = None,
                                 init_mode: str = "noisy", pose_lr: float = 1e-4, pose_opt_delay: int = 1000,
                                 learn_rotation: bool = True, learn_translation: bool = True,
                                 rotation_reg_weight: float = 0.01, translation_reg_weight: float = 0.001, *,
                                 train_data: Optional[BlenderData] = None, val_data: Optional[BlenderData] = None,
                                 process_group=None, experiment_name: Optional[str] = None,
                                 log=print) -> Dict[str, object]:
    """Reference train_pose_opt.py:613-1054 (same arguments, outputs and files).
    ``train_data`` / ``val_data`` (optional) replace the on-disk scene; ``process_group``
    makes it data parallel; ``experiment_name`` pins the generated run name (all ranks)."""
    import torch.distributed as dist

    rank, world = 0, 1
    if process_group is not None:
        rank, world = dist.get_rank(process_group), dist.get_world_size(process_group)
    check_run_args(config, world, train_data, val_data)
    set_seed(config.train.seed)
    device = config.train.device
    if device.startswith("cuda") and not torch.cuda.is_available():
        raise RuntimeError("noisy_src.train_pose_opt needs a ROCm device (no CPU path)")
    exp_name = experiment_name or generate_experiment_name(config.data.scene_name, noise_config, init_mode)
    output_dir = Path(config.train.output_dir) / exp_name
    logger = ExperimentLogger(output_dir, exp_name, use_tensorboard=True) if rank == 0 else None
    if logger is not None:
        logger.log_config(config)
    if train_data is None:
        root = config.data.data_root if config.data.data_root is not None else Path("data") / "raw"
        train_data = load_blender_data(root, config.data.scene_name, "train", config.data.img_scale, device)
        val_data = load_blender_data(root, config.data.scene_name, "val", config.data.img_scale, device)
    gt_train_poses = train_data.poses.clone()
    if init_mode == "noisy" and noise_config is not None and noise_config.has_noise:
        initial_poses, _ = add_noise_to_poses(train_data.poses, noise_config)
        if logger is not None:
            errs = [compute_pose_error(gt_train_poses[i].cpu(), initial_poses[i].cpu())
                    for i in range(len(initial_poses))]
            log(f"initial pose errors: rotation {np.mean([e['rotation_error_deg'] for e in errs]):.3f} deg, "
                f"translation {np.mean([e['translation_error'] for e in errs]):.4f}")
    else:
        initial_poses = gt_train_poses.clone()
    camera_params = CameraPoseParameters(initial_poses, learn_rotation, learn_translation).to(device)
    model_coarse, model_fine = create_nerf_for(config, device)
    if logger is not None:
        logger.log_model_info(model_coarse, "model_coarse")
        if model_fine is not None:
            logger.log_model_info(model_fine, "model_fine")
    _, pixel_sampler = create_pixel_dataset(train_data)
    pixel_sampler.batch_size = config.data.batch_size
    trainer = PoseTrainer(model_coarse, model_fine, camera_params, pixel_sampler, config.render, lr=config.train.lr,
                          pose_lr=pose_lr, lr_decay=config.train.lr_decay, rotation_reg_weight=rotation_reg_weight,
                          translation_reg_weight=translation_reg_weight, process_group=process_group)
    optimizer_nerf, optimizer_poses = trainer.optimizer_nerf, trainer.optimizer_poses
    lpips_metric = LPIPSMetric(device=device) if rank == 0 else None
    if lpips_metric is not None and not lpips_metric.available:
        lpips_metric = None
    if rank == 0:
        nc = noise_config
        (output_dir / "experiment_config.json").write_text(json.dumps({
            "scene": config.data.scene_name, "experiment_name": exp_name, "init_mode": init_mode,
            "pose_optimization": {"learn_rotation": learn_rotation, "learn_translation": learn_translation,
                                  "pose_lr": pose_lr, "pose_opt_delay": pose_opt_delay,
                                  "rotation_reg_weight": rotation_reg_weight,
                                  "translation_reg_weight": translation_reg_weight},
            "noise_config": {"rotation_noise_deg": nc.rotation_noise_deg, "translation_noise": nc.translation_noise,
                             "translation_noise_pct": nc.translation_noise_pct, "seed": nc.seed,
                             "has_noise": nc.has_noise} if nc else None,
            "num_iterations": config.train.num_iterations, "batch_size": config.data.batch_size,
            "timestamp": datetime.now().isoformat(), "data_parallel_ranks": world}, indent=2))
        log(f"joint NeRF + pose optimisation: {exp_name} -> {output_dir} ({world} rank(s))")

    B = config.data.batch_size
    rc = config.render
    val_idx = torch.arange(val_data.images.shape[0], device=device)
    start = time.time()
    best_psnr = 0.0
    lagged = LaggedScalars()  # logged losses read one iteration late: no per-step host sync
    t_prev = time.time()

    def log_iteration(done):
        if done is None or logger is None:
            return
        vals, (it, keys, lr, now, batch_time) = done
        vm = dict(zip(keys, vals))
        last = vm.get("loss_fine", vm["loss_coarse"])
        psnr = -10.0 * math.log10(last) if last > 0 else float("inf")
        logger.log_training(TrainingMetrics(iteration=it, loss=vm["loss"], loss_coarse=vm["loss_coarse"],
                                            loss_fine=vm.get("loss_fine"), psnr=psnr, learning_rate=lr,
                                            time_per_iter=batch_time, rays_per_sec=B / batch_time))
        if it % config.train.log_every == 0:
            log(f"[{it:7d}/{config.train.num_iterations}] loss: {vm['loss']:.5f} | psnr: {psnr:.2f} | "
                f"lr: {lr:.2e} | poses: {'optimizing' if now else 'frozen'} | "
                f"time: {(time.time() - start) / 60:.1f}min")

    for iteration in range(config.train.num_iterations):
        batch = pixel_sampler.sample_batch()  # the global batch, identical on every rank
        now = iteration >= pose_opt_delay
        t_rand = torch.rand(B, rc.num_samples, device=device) if rc.perturb else None
        u = torch.rand(B, rc.num_samples_fine, device=device) if (rc.use_hierarchical and model_fine) else None
        sl = rank_slice(B, rank, world) if world > 1 else slice(0, B)
        m = trainer.step(batch.slice(sl) if world > 1 else batch, optimize_poses=now,
                         t_rand=None if t_rand is None else t_rand[sl], u=None if u is None else u[sl])
        keys = ["loss", "loss_coarse"] + (["loss_fine"] if "loss_fine" in m else [])
        t_now = time.time()
        log_iteration(lagged.push(mean_over_ranks([m[k] for k in keys], process_group),
                                  (iteration, keys, optimizer_nerf.param_groups[0]["lr"], now, t_now - t_prev)))
        t_prev = t_now
        if logger is None:
            continue
        if iteration > 0 and (iteration % config.train.val_every == 0 or iteration % config.train.save_every == 0):
            log_iteration(lagged.flush())
        if iteration % config.train.val_every == 0 and iteration > 0:
            pe = camera_params.compute_pose_errors(gt_train_poses)
            vmx = evaluate_with_poses(model_coarse, model_fine, camera_params, val_data, val_idx, rc, logger,
                                      iteration, num_images=5, lpips_metric=lpips_metric)
            logger.log_validation(vmx)
            is_best = vmx.psnr > best_psnr
            best_psnr = max(best_psnr, vmx.psnr)
            log(f"  validation @ {iteration}: PSNR {vmx.psnr:.2f} dB; pose error rot "
                f"{pe['rotation_error_mean']:.3f} deg, trans {pe['translation_error_mean']:.4f}")
            save_checkpoint_with_poses(output_dir, iteration, model_coarse, model_fine, camera_params,
                                       optimizer_nerf, optimizer_poses, config, noise_config,
                                       metrics={"psnr": vmx.psnr, "ssim": vmx.ssim}, pose_errors=pe,
                                       is_best=is_best)
            t_prev = time.time()  # the next iteration's time excludes the validation
        elif iteration % config.train.save_every == 0 and iteration > 0:
            pe = camera_params.compute_pose_errors(gt_train_poses)
            save_checkpoint_with_poses(output_dir, iteration, model_coarse, model_fine, camera_params,
                                       optimizer_nerf, optimizer_poses, config, noise_config, pose_errors=pe)
            t_prev = time.time()
    log_iteration(lagged.flush())
    result = {"model_coarse": model_coarse, "model_fine": model_fine, "camera_params": camera_params,
              "output_dir": output_dir, "pose_errors": camera_params.compute_pose_errors(gt_train_poses)}
    if logger is not None:
        final_pe = result["pose_errors"]
        final = evaluate_with_poses(model_coarse, model_fine, camera_params, val_data, val_idx, rc, logger,
                                    config.train.num_iterations, num_images=val_data.images.shape[0],
                                    lpips_metric=lpips_metric)
        # (the reference does not write the final evaluation to val_metrics.csv, :1002-1019)
        save_checkpoint_with_poses(output_dir, config.train.num_iterations, model_coarse, model_fine, camera_params,
                                   optimizer_nerf, optimizer_poses, config, noise_config,
                                   metrics={"psnr": final.psnr, "ssim": final.ssim}, pose_errors=final_pe)
        with torch.no_grad():
            final_poses = camera_params.get_all_poses()
        torch.save({"initial_poses": camera_params.initial_poses.cpu(), "optimized_poses": final_poses.cpu(),
                    "ground_truth_poses": gt_train_poses.cpu(), "pose_errors": final_pe},
                   output_dir / "final_poses.pt")
        logger.save_summary()
        logger.close()
        log(f"final: PSNR {final.psnr:.2f} dB; pose error rot {final_pe['rotation_error_mean']:.3f} deg, "
            f"trans {final_pe['translation_error_mean']:.4f}; results in {output_dir}")
        result["val"] = final
    if process_group is not None:
        dist.barrier(process_group)
    return result


def create_nerf_for(config: NeRFConfig, device):
    """create_nerf + .to(device); no fine network without hierarchical sampling
    (train_pose_opt.py:772-777)."""
    from .model import create_nerf
    mc, mf = create_nerf(config.model)
    mc = mc.to(device)
    mf = mf.to(device) if config.render.use_hierarchical else None
    return mc, mf


def build_arg_parser():
    """Reference train_pose_opt.py:1057-1142 flags (same names and defaults) plus ``--precision``."""
    import argparse
    ap = argparse.ArgumentParser(description="Joint NeRF + camera pose optimisation (MI355X HIP path)")
    ap.add_argument("--scene", type=str, default="lego")
    ap.add_argument("--data_root", type=str, default=None)
    ap.add_argument("--img_scale", type=float, default=0.5)
    ap.add_argument("--batch_size", type=int, default=1024, help="global batch (pixels) over all ranks")
    ap.add_argument("--num_iters", type=int, default=50000)
    ap.add_argument("--lr", type=float, default=5e-4)
    ap.add_argument("--init_mode", type=str, default="noisy", choices=["noisy", "clean"])
    ap.add_argument("--pose_lr", type=float, default=1e-4)
    ap.add_argument("--pose_opt_delay", type=int, default=1000)
    ap.add_argument("--no_learn_rotation", action="store_true")
    ap.add_argument("--no_learn_translation", action="store_true")
    ap.add_argument("--rotation_reg_weight", type=float, default=0.01)
    ap.add_argument("--translation_reg_weight", type=float, default=0.001)
    ap.add_argument("--rotation_noise", type=float, default=0.0)
    ap.add_argument("--translation_noise", type=float, default=0.0)
    ap.add_argument("--translation_noise_pct", type=float, default=0.0)
    ap.add_argument("--noise_seed", type=int, default=None)
    ap.add_argument("--no_hierarchical", action="store_true")
    ap.add_argument("--num_samples", type=int, default=64)
    ap.add_argument("--num_samples_fine", type=int, default=128)
    ap.add_argument("--log_every", type=int, default=100)
    ap.add_argument("--val_every", type=int, default=2500)
    ap.add_argument("--save_every", type=int, default=10000)
    ap.add_argument("--output_dir", type=str, default="outputs")
    ap.add_argument("--device", type=str, default="cuda")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--precision", type=str, default="fp32", choices=["fp32", "bf16", "fp16"],
                    help="MLP operand precision (fp32 = the reference's numerics)")
    return ap


def main(argv=None) -> None:
    """``python -m noisy_src.train_pose_opt`` (or under ``torchrun`` for data parallelism)."""
    from .config import DataConfig, ModelConfig, TrainConfig

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
        train=TrainConfig(lr=a.lr, num_iterations=a.num_iters, output_dir=Path(a.output_dir), device=device,
                          seed=a.seed, log_every=a.log_every, val_every=a.val_every, save_every=a.save_every))
    name = [generate_experiment_name(a.scene, noise_config, a.init_mode)]
    if pg is not None:
        import torch.distributed as dist
        dist.broadcast_object_list(name, src=0, group=pg)
    train_with_pose_optimization(cfg, noise_config, a.init_mode, a.pose_lr, a.pose_opt_delay,
                                 not a.no_learn_rotation, not a.no_learn_translation, a.rotation_reg_weight,
                                 a.translation_reg_weight, process_group=pg, experiment_name=name[0])
    if pg is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


__all__ = ["set_seed", "CameraPoseParameters", "train_step_with_poses", "render_image_with_pose",
           "evaluate_with_poses", "save_checkpoint_with_poses", "generate_experiment_name",
           "train_with_pose_optimization", "main"]

if __name__ == "__main__":
    main()
