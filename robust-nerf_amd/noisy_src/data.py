"""
Scene data and ray batches — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src/data.py``.

* ``load_blender_data`` restates the reference's image preprocessing (data.py:50-158):
  RGBA composited on white and re-quantised to uint8, LANCZOS resize, focal from the
  resized width.  The NeRF synthetic dataset is not in this image (no network); the
  loader works on any directory laid out like it, and ``synthetic_blender_data``
  builds a same-shaped scene (reference GT poses, random images) for the benchmark.
* ``RayDataset`` builds the ray table on the device with the HIP ``get_rays`` kernel
  (data.py:161-261; 100 x 640k rays x 36 B = 2.3 GB at 800^2, resident in HBM).
* ``RaySampler`` keeps the reference's epoch ``randperm`` sampler (data.py:264-321)
  with the permutation on the device and the batch assembled by one HIP gather of
  the ray table (``nr_gather_rays``): no host work per batch.
"""

from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from . import ops
from .config import DataConfig
from .noise import NoiseConfig, add_noise_to_pose, set_noise_seed


@dataclass
class BlenderData:
    """Reference data.py:26-47: images (N,H,W,3) in [0,1], poses (N,4,4), H, W, focal."""

    images: torch.Tensor
    poses: torch.Tensor
    H: int
    W: int
    focal: float


def load_blender_data(data_root: Path, scene_name: str, split: str = "train", img_scale: float = 0.5,
                      device: str = "cpu") -> BlenderData:
    """Reference data.py:50-158."""
    from PIL import Image

    data_root = Path(data_root)
    scene_dir = None
    for cand in (data_root / scene_name, data_root / "nerf_synthetic" / scene_name):
        if cand.exists():
            scene_dir = cand
            break
    if scene_dir is None:
        raise FileNotFoundError(f"Could not find scene '{scene_name}' in {data_root}")
    tpath = scene_dir / f"transforms_{split}.json"
    if not tpath.exists():
        raise FileNotFoundError(f"Missing transforms file: {tpath}")
    meta = json.loads(tpath.read_text())
    camera_angle_x = float(meta["camera_angle_x"])
    images, poses = [], []
    for frame in meta["frames"]:
        img_path = scene_dir / f"{frame['file_path']}.png"
        if not img_path.exists():
            raise FileNotFoundError(f"Missing image: {img_path}")
        img = Image.open(img_path)
        if img.mode == "RGBA":
            arr = np.array(img, dtype=np.float32) / 255.0
            rgb = arr[..., :3] * arr[..., 3:4] + (1.0 - arr[..., 3:4])
            img = Image.fromarray((rgb * 255).astype(np.uint8))
        else:
            img = img.convert("RGB")
        w0, h0 = img.size
        if img_scale != 1.0:
            img = img.resize((int(w0 * img_scale), int(h0 * img_scale)), Image.LANCZOS)
        images.append(torch.from_numpy(np.array(img, dtype=np.float32) / 255.0))
        poses.append(torch.from_numpy(np.array(frame["transform_matrix"], dtype=np.float32)))
    images = torch.stack(images, 0)
    poses = torch.stack(poses, 0)
    H, W = images.shape[1:3]
    focal = 0.5 * W / np.tan(0.5 * camera_angle_x)
    return BlenderData(images=images.to(device), poses=poses.to(device), H=H, W=W, focal=float(focal))


# lego transforms_*.json camera_angle_x (the synthetic scenes share it)
LEGO_CAMERA_ANGLE_X = 0.6911112070083618


def synthetic_blender_data(poses: torch.Tensor, H: int = 800, W: int = 800,
                           camera_angle_x: float = LEGO_CAMERA_ANGLE_X, seed: int = 0,
                           device="cuda") -> BlenderData:
    """A scene shaped like the reference's (real poses, H x W images in [0,1]) with
    random pixels: the dataset itself is not available offline."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    images = torch.rand(poses.shape[0], H, W, 3, generator=g).to(device)
    focal = 0.5 * W / np.tan(0.5 * camera_angle_x)
    return BlenderData(images=images, poses=poses.to(device=device, dtype=torch.float32), H=H, W=W,
                       focal=float(focal))


class RayDataset:
    """Reference data.py:161-261: every ray of every training image, precomputed on the
    device (HIP ``nr_ray_directions`` + ``nr_get_rays``), optionally from noisy poses."""

    def __init__(self, data: BlenderData, batch_size: int = 1024, noise_config: Optional[NoiseConfig] = None):
        self.H, self.W, self.focal = data.H, data.W, data.focal
        self.noise_config = noise_config
        self.original_poses = data.poses.clone()
        dev = data.images.device
        self.directions = ops.ray_directions(data.H, data.W, data.focal, data.W / 2.0, data.H / 2.0, dev)
        if noise_config is not None and noise_config.seed is not None:
            set_noise_seed(noise_config.seed)
        n = data.images.shape[0]
        hw = data.H * data.W
        self.rays_o = torch.empty(n * hw, 3, device=dev)
        self.rays_d = torch.empty(n * hw, 3, device=dev)
        self.noise_info = []
        for i in range(n):
            pose = data.poses[i]
            if noise_config is not None and noise_config.has_noise:
                dist = torch.norm(pose[:3, 3]).item()
                pose, info = add_noise_to_pose(pose, rotation_noise_deg=noise_config.rotation_noise_deg,
                                               translation_noise=noise_config.get_translation_std(dist))
                self.noise_info.append(info)
            o, d = ops.get_rays(self.directions, pose.contiguous())
            self.rays_o[i * hw:(i + 1) * hw] = o.reshape(-1, 3)
            self.rays_d[i * hw:(i + 1) * hw] = d.reshape(-1, 3)
        self.colors = data.images.reshape(-1, 3)
        self.n_rays = self.rays_o.shape[0]
        if not self.noise_info:
            self.noise_info = None

    def __len__(self) -> int:
        return self.n_rays

    def __getitem__(self, idx):
        return {"rays_o": self.rays_o[idx], "rays_d": self.rays_d[idx], "target_rgb": self.colors[idx]}


class RaySampler:
    """Reference data.py:264-321: epoch iteration over a device ``randperm`` (or arange),
    and ``sample_batch`` with replacement."""

    def __init__(self, dataset: RayDataset, batch_size: int = 1024, shuffle: bool = True):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.device = dataset.rays_o.device
        self.n_rays = dataset.n_rays
        self._reset_indices()

    def _reset_indices(self) -> None:
        if self.shuffle:
            self.indices = torch.randperm(self.n_rays, device=self.device)
        else:
            self.indices = torch.arange(self.n_rays, device=self.device)
        self.current_idx = 0

    def __iter__(self) -> Iterator[dict]:
        self._reset_indices()
        return self

    def _gather(self, idx: torch.Tensor, validate: bool = False) -> dict:
        ds = self.dataset
        o, d, rgb = ops.gather_rays(idx, ds.rays_o, ds.rays_d, ds.colors, validate=validate)
        return {"rays_o": o, "rays_d": d, "target_rgb": rgb}

    def get_batch(self, indices: torch.Tensor) -> dict:
        """The batch of caller-chosen ray indices (the reference's ``rays_o[batch_indices]``
        ..., data.py:305-309): one gather launch in its validating mode, so an index
        outside the table raises IndexError as torch indexing does.  The sampler's own
        draws (randperm / randint) are in range by construction and skip the check."""
        return self._gather(indices.to(self.device), validate=True)

    def __next__(self) -> dict:
        if self.current_idx >= self.n_rays:
            raise StopIteration
        end = min(self.current_idx + self.batch_size, self.n_rays)
        idx = self.indices[self.current_idx:end]
        self.current_idx = end
        return self._gather(idx)

    def __len__(self) -> int:
        return (self.n_rays + self.batch_size - 1) // self.batch_size

    def sample_batch(self) -> dict:
        return self._gather(torch.randint(0, self.n_rays, (self.batch_size,), device=self.device))


def create_data_loaders(config: DataConfig, device: str = "cpu",
                        noise_config: Optional[NoiseConfig] = None) -> Tuple[RaySampler, BlenderData, BlenderData]:
    """Reference data.py:324-383: (train sampler, train data, val data)."""
    data_root = config.data_root
    if data_root is None:
        data_root = Path("data") / "raw"
    train = load_blender_data(data_root, config.scene_name, "train", config.img_scale, device)
    val = load_blender_data(data_root, config.scene_name, "val", config.img_scale, device)
    ds = RayDataset(train, batch_size=config.batch_size, noise_config=noise_config)
    return RaySampler(ds, batch_size=config.batch_size, shuffle=config.shuffle), train, val
