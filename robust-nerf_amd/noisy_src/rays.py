"""
Ray generation and sampling — drop-in for ShawnnnLiu/Robust-NeRF
``noisy_src/rays.py`` (same function names, arguments and results), computed by
the HIP kernels of csrc/rays.hip and csrc/sampling.hip.

The random draws the reference makes with ``torch.rand`` (stratified jitter at
rays.py:204, inverse-CDF uniforms at rays.py:255) are drawn the same way here
unless the caller injects them (``t_rand=`` / ``u=``), which the parity tests
use to compare against the oracle on identical inputs.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import ops


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("noisy_src HIP path needs a ROCm device; there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def get_ray_directions(H: int, W: int, focal: float, center: Tuple[float, float] | None = None,
                       device=None) -> torch.Tensor:
    """Reference rays.py:17-64 -> (H, W, 3) on the ROCm device."""
    if center is None:
        cx, cy = W / 2.0, H / 2.0
    else:
        cx, cy = center
    return ops.ray_directions(H, W, focal, cx, cy, device or _default_device())


def get_rays(directions: torch.Tensor, c2w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference rays.py:67-99 -> (rays_o, rays_d), rays_d normalised; differentiable
    w.r.t. c2w (and the directions), as data_pose_opt.py:83-148 relies on."""
    if directions.device != c2w.device:
        directions = directions.to(c2w.device)
    return ops.get_rays(directions, c2w)


def get_rays_batch(H: int, W: int, focal: float, c2w_batch: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference rays.py:102-142 -> (N, H, W, 3) each."""
    directions = get_ray_directions(H, W, focal, device=c2w_batch.device)
    outs = [get_rays(directions, c2w_batch[i]) for i in range(c2w_batch.shape[0])]
    return torch.stack([o for o, _ in outs]), torch.stack([d for _, d in outs])


def sample_along_rays(rays_o: torch.Tensor, rays_d: torch.Tensor, near: float, far: float, num_samples: int,
                      perturb: bool = True, lindisp: bool = False,
                      t_rand: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference rays.py:145-210 -> (pts (..., N, 3), z_vals (..., N))."""
    batch_shape = rays_o.shape[:-1]
    ro = rays_o.reshape(-1, 3)
    rd = rays_d.reshape(-1, 3)
    if perturb and t_rand is None:
        t_rand = torch.rand(*batch_shape, num_samples, device=rays_o.device)
    tr = t_rand.reshape(-1, num_samples) if perturb else None
    pts, z = ops.stratified_sample(ro, rd, near, far, num_samples, t_rand=tr, lindisp=lindisp)
    return pts.reshape(*batch_shape, num_samples, 3), z.reshape(*batch_shape, num_samples)


def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, num_samples: int, det: bool = False,
               u: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Reference rays.py:213-279 -> samples (..., num_samples)."""
    if not det and u is None:
        u = torch.rand(*bins.shape[:-1], num_samples, device=weights.device)
    return ops.sample_pdf(bins, weights, num_samples, u=None if det else u)


def sample_hierarchical(rays_o: torch.Tensor, rays_d: torch.Tensor, z_vals: torch.Tensor, weights: torch.Tensor,
                        num_samples_fine: int, det: bool = False,
                        u: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference rays.py:282-333 -> (pts_fine (..., Nc+Nf, 3), z_vals_fine (..., Nc+Nf)), sorted."""
    batch_shape = rays_o.shape[:-1]
    Nc = z_vals.shape[-1]
    if not det and u is None:
        u = torch.rand(*batch_shape, num_samples_fine, device=z_vals.device)
    pts, z = ops.sample_hierarchical(rays_o.reshape(-1, 3), rays_d.reshape(-1, 3), z_vals.reshape(-1, Nc),
                                     weights.reshape(-1, Nc), num_samples_fine,
                                     u=None if det else u.reshape(-1, num_samples_fine))
    T = Nc + num_samples_fine
    return pts.reshape(*batch_shape, T, 3), z.reshape(*batch_shape, T)
