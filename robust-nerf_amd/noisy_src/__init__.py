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

__all__ = [
    "NeRFConfig", "ModelConfig", "RenderConfig", "DataConfig", "TrainConfig", "PoseOptConfig",
    "NeRF", "PositionalEncoding", "create_nerf",
    "NeRFRenderer", "render_rays", "raw2outputs",
    "get_ray_directions", "get_rays", "get_rays_batch", "sample_along_rays", "sample_pdf", "sample_hierarchical",
]
