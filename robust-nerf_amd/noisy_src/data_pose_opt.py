"""
Pixel batches for joint pose optimisation — drop-in for ShawnnnLiu/Robust-NeRF
``noisy_src/data_pose_opt.py``.

The reference regenerates each batch's rays from the current (learnable) poses with a
Python loop over the unique images of the batch, two ``.item()`` syncs per image and
masked scatters (data_pose_opt.py:83-148).  Here one HIP kernel
(``nr_rays_from_pixels_fwd``) gathers every ray straight from (image, u, v) and its
image's pose, and its backward scatters dL/d(rays_o, rays_d) into dL/d(poses): same
values, same gradient, no host round trips.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch

from . import ops
from .data import BlenderData


@dataclass
class PixelBatch:
    """Reference data_pose_opt.py:21-26."""

    image_indices: torch.Tensor  # (B,) int64
    pixel_coords: torch.Tensor   # (B, 2) float (u, v)
    target_rgb: torch.Tensor     # (B, 3)
    # set by PixelSampler.sample_batch, whose indices are in range by construction;
    # batches built elsewhere are validated (one host sync) before the ray kernel
    in_range: bool = False

    def slice(self, sl: slice) -> "PixelBatch":
        """Rows ``sl`` of the batch (a data-parallel rank's contiguous share)."""
        return PixelBatch(self.image_indices[sl], self.pixel_coords[sl], self.target_rgb[sl], self.in_range)


class PixelDataset:
    """Reference data_pose_opt.py:29-148."""

    def __init__(self, data: BlenderData):
        self.H, self.W, self.focal = data.H, data.W, data.focal
        self.device = data.images.device
        n_img = data.images.shape[0]
        hw = self.H * self.W
        v, u = torch.meshgrid(torch.arange(self.H, dtype=torch.float32, device=self.device),
                              torch.arange(self.W, dtype=torch.float32, device=self.device), indexing="ij")
        single = torch.stack([u.flatten(), v.flatten()], dim=-1)
        self.image_indices = torch.repeat_interleave(torch.arange(n_img, dtype=torch.long, device=self.device), hw)
        self.pixel_coords = single.unsqueeze(0).expand(n_img, -1, -1).reshape(-1, 2)
        self.target_rgb = data.images.reshape(-1, 3)
        self.n_pixels = n_img * hw
        self.ray_directions = ops.ray_directions(self.H, self.W, self.focal, self.W / 2.0, self.H / 2.0, self.device)

    def get_rays_from_pixels(self, pixel_batch: PixelBatch, poses: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Reference data_pose_opt.py:83-148.  ``poses`` holds one pose per UNIQUE image of
        the batch, in ascending image order (``poses_all[torch.unique(indices)]``)."""
        uniq, inv = torch.unique(pixel_batch.image_indices, return_inverse=True)
        if poses.shape[0] != uniq.shape[0]:
            raise ValueError(f"get_rays_from_pixels: {poses.shape[0]} poses for {uniq.shape[0]} unique images")
        # ``inv`` indexes ``uniq`` by construction: nothing to validate here
        return ops.rays_from_pixels(inv, pixel_batch.pixel_coords, poses, self.H, self.W, self.focal, validate=False)


class PixelSampler:
    """Reference data_pose_opt.py:151-223: uniform pixels with replacement."""

    def __init__(self, dataset: PixelDataset, batch_size: int = 1024):
        self.dataset = dataset
        self.batch_size = batch_size
        self.device = dataset.device
        self.n_pixels = dataset.n_pixels

    def sample_batch(self, generator=None) -> PixelBatch:
        """``generator`` (optional, on the dataset's device) makes the draw reproducible
        across data-parallel ranks that each take a slice of it."""
        idx = torch.randint(0, self.n_pixels, (self.batch_size,), device=self.device, generator=generator)
        ds = self.dataset
        return PixelBatch(image_indices=ds.image_indices[idx], pixel_coords=ds.pixel_coords[idx],
                          target_rgb=ds.target_rgb[idx], in_range=True)

    def get_rays_for_batch(self, pixel_batch: PixelBatch, poses: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Reference data_pose_opt.py:200-223 with ``poses`` = every image's pose (N,4,4):
        the kernel indexes them by image directly (the reference's unique/select/loop
        gives the same rays), and the pose gradient lands on every image in the batch."""
        ds = self.dataset
        return ops.rays_from_pixels(pixel_batch.image_indices, pixel_batch.pixel_coords, poses, ds.H, ds.W, ds.focal,
                                    validate=not pixel_batch.in_range)


def create_pixel_dataset(data: BlenderData) -> Tuple[PixelDataset, PixelSampler]:
    """Reference data_pose_opt.py:226-241."""
    ds = PixelDataset(data)
    return ds, PixelSampler(ds)
