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
"""

from __future__ import annotations

import random
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .config import RenderConfig
from .data import BlenderData
from .data_pose_opt import PixelBatch, PixelSampler
from .metrics import compute_mse, compute_psnr, compute_ssim
from .model import NeRF
from .noise import compute_pose_error
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
                        logger=None, iteration: int = 0, num_images: int = 5, lpips_metric=None) -> Dict[str, object]:
    """Reference train_pose_opt.py:474-545: renders the first ``num_images`` validation
    views from their GROUND-TRUTH poses; returns the mean metrics and the per-image lists."""
    psnr, ssim, mse = [], [], []
    for idx in val_indices[:min(num_images, len(val_indices))]:
        out = render_image_with_pose(model_coarse, model_fine, val_data.poses[idx], val_data.H, val_data.W,
                                     val_data.focal, render_config)
        pred, target = out["rgb"], val_data.images[idx]
        mse.append(compute_mse(pred, target).item())
        psnr.append(compute_psnr(pred, target).item())
        ssim.append(compute_ssim(pred, target).item())
    return {"iteration": iteration, "psnr": float(np.mean(psnr)), "ssim": float(np.mean(ssim)),
            "mse": float(np.mean(mse)), "lpips": None, "per_image_psnr": psnr, "per_image_ssim": ssim}


def train_with_pose_optimization(config, train_data: BlenderData, val_data: Optional[BlenderData] = None,
                                 init_mode: str = "noisy", noise_config=None, pose_lr: float = 1e-4,
                                 pose_opt_delay: int = 1000, learn_rotation: bool = True,
                                 learn_translation: bool = True, rotation_reg_weight: float = 0.01,
                                 translation_reg_weight: float = 0.001, logger=None, log=print) -> Dict[str, object]:
    """Reference train_pose_opt.py:613-1054 without the image/checkpoint I/O: seeds, noisy
    (or clean) initial poses, CameraPoseParameters, both networks, NeRF and pose Adams
    (fused) with their LambdaLRs (the pose one steps only once poses optimise), the
    pixel sampler, and train_step_with_poses every iteration."""
    import time

    from .data_pose_opt import create_pixel_dataset
    from .engine import lr_lambda_factory
    from .logger import TrainingMetrics
    from .model import create_nerf
    from .noise import add_noise_to_poses

    set_seed(config.train.seed)
    dev = train_data.images.device
    gt = train_data.poses.clone()
    if init_mode == "noisy" and noise_config is not None and noise_config.has_noise:
        init, _ = add_noise_to_poses(train_data.poses, noise_config)
    else:
        init = gt.clone()
    cam = CameraPoseParameters(init, learn_rotation, learn_translation).to(dev)
    mc, mf = create_nerf(config.model)
    mc = mc.to(dev)
    mf = mf.to(dev) if config.render.use_hierarchical else None
    nerf_params = list(mc.parameters()) + (list(mf.parameters()) if mf is not None else [])
    opt_n = FusedAdam(nerf_params, lr=config.train.lr)
    opt_p = FusedAdam(cam.parameters(), lr=pose_lr)
    lam = lr_lambda_factory(config.train.lr_decay)
    sch_n = torch.optim.lr_scheduler.LambdaLR(opt_n, lam)
    sch_p = torch.optim.lr_scheduler.LambdaLR(opt_p, lam)
    _, sampler = create_pixel_dataset(train_data)
    sampler.batch_size = config.data.batch_size
    t0 = time.time()
    for it in range(config.train.num_iterations):
        batch = sampler.sample_batch()
        now = it >= pose_opt_delay
        tb = time.time()
        m = train_step_with_poses(mc, mf, cam, sampler, opt_n, opt_p if now else None, batch, config.render,
                                  optimize_poses=now, rotation_reg_weight=rotation_reg_weight,
                                  translation_reg_weight=translation_reg_weight)
        sch_n.step()
        if now:
            sch_p.step()
        dt = time.time() - tb
        if logger is not None:
            logger.log_training(TrainingMetrics(iteration=it, loss=m["loss"], loss_coarse=m["loss_coarse"],
                                                loss_fine=m.get("loss_fine"), psnr=m["psnr"],
                                                learning_rate=opt_n.param_groups[0]["lr"], time_per_iter=dt,
                                                rays_per_sec=config.data.batch_size / dt))
        if it % config.train.log_every == 0:
            log(f"iter {it}: loss {m['loss']:.5f} psnr {m['psnr']:.2f} poses {'on' if now else 'frozen'} "
                f"({time.time() - t0:.1f} s)")
    out = {"model_coarse": mc, "model_fine": mf, "camera_params": cam,
           "pose_errors": cam.compute_pose_errors(gt)}
    if val_data is not None:
        out["val"] = evaluate_with_poses(mc, mf, cam, val_data, torch.arange(val_data.images.shape[0]), config.render)
    return out


def main(argv=None) -> None:
    """``python -m noisy_src.train_pose_opt`` — the reference CLI (train_pose_opt.py:1057-1190),
    same flags plus ``--precision``; needs the NeRF synthetic scene under ``--data_root``."""
    import argparse
    from pathlib import Path

    from .config import DataConfig, ModelConfig, NeRFConfig, TrainConfig
    from .data import load_blender_data
    from .logger import ExperimentLogger
    from .noise import NoiseConfig

    ap = argparse.ArgumentParser(description="Joint NeRF + camera pose optimisation (MI355X HIP path)")
    ap.add_argument("--scene", type=str, default="lego")
    ap.add_argument("--data_root", type=str, default=None)
    ap.add_argument("--img_scale", type=float, default=0.5)
    ap.add_argument("--batch_size", type=int, default=1024)
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
    ap.add_argument("--output_dir", type=str, default="outputs")
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
        train=TrainConfig(lr=a.lr, num_iterations=a.num_iters, log_every=a.log_every,
                          output_dir=Path(a.output_dir), device=a.device, seed=a.seed))
    noise = NoiseConfig(rotation_noise_deg=a.rotation_noise, translation_noise=a.translation_noise,
                        translation_noise_pct=a.translation_noise_pct, seed=a.noise_seed)
    root = cfg.data.data_root or Path("data") / "raw"
    train_data = load_blender_data(root, a.scene, "train", a.img_scale, a.device)
    val_data = load_blender_data(root, a.scene, "val", a.img_scale, a.device)
    import time
    name = f"{a.scene}_poseopt_{a.init_mode}init_{noise}_{time.strftime('%Y%m%d_%H%M%S')}"  # (:274-287)
    logger = ExperimentLogger(Path(a.output_dir) / name, name)
    logger.log_config(cfg)
    train_with_pose_optimization(cfg, train_data, val_data, a.init_mode, noise, a.pose_lr, a.pose_opt_delay,
                                 not a.no_learn_rotation, not a.no_learn_translation, a.rotation_reg_weight,
                                 a.translation_reg_weight, logger=logger)
    logger.close()


if __name__ == "__main__":
    main()
