"""
Robust-NeRF on MI355X — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src``
(reference noisy_src/__init__.py:10-66).

The hot path (rays.py, model.py, rendering.py, the SE(3) pose path and the
optimizer tail) runs as hand-written gfx950 HIP kernels behind the C ABI in
include/nerf_hip.h; see DESIGN.md.
"""

__version__ = "0.1.0"

from .config import NeRFConfig, ModelConfig, RenderConfig, DataConfig, TrainConfig, PoseOptConfig
from .model import NeRF, PositionalEncoding, create_nerf
from .rendering import NeRFRenderer, render_rays, raw2outputs
from .rays import (
    get_ray_directions,
    get_rays,
    get_rays_batch,
    sample_along_rays,
    sample_pdf,
    sample_hierarchical,
)
from .data import BlenderData, load_blender_data, RayDataset, RaySampler, create_data_loaders
from .data_pose_opt import PixelBatch, PixelDataset, PixelSampler, create_pixel_dataset
from .train import train, train_step, render_image
from .train_pose_opt import CameraPoseParameters, train_step_with_poses, render_image_with_pose
from .metrics import compute_psnr, compute_ssim, compute_mse, compute_all_metrics
from .logger import ExperimentLogger, TrainingMetrics, ValidationMetrics
from .noise import NoiseConfig, add_noise_to_pose, add_noise_to_poses, compute_pose_error

__all__ = [
    "NeRFConfig", "ModelConfig", "RenderConfig", "DataConfig", "TrainConfig", "PoseOptConfig",
    "NeRF", "PositionalEncoding", "create_nerf",
    "NeRFRenderer", "render_rays", "raw2outputs",
    "get_ray_directions", "get_rays", "get_rays_batch", "sample_along_rays", "sample_pdf", "sample_hierarchical",
    "BlenderData", "load_blender_data", "RayDataset", "RaySampler", "create_data_loaders",
    "PixelBatch", "PixelDataset", "PixelSampler", "create_pixel_dataset",
    "train", "train_step", "render_image",
    "CameraPoseParameters", "train_step_with_poses", "render_image_with_pose",
    "compute_psnr", "compute_ssim", "compute_mse", "compute_all_metrics",
    "ExperimentLogger", "TrainingMetrics", "ValidationMetrics",
    "NoiseConfig", "add_noise_to_pose", "add_noise_to_poses", "compute_pose_error",
]
