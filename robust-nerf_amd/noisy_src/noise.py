"""
Camera-pose noise — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src/noise.py``.

Produces the noisy initial poses of BASELINE cfg #3 (5 deg rotation + 5 % translation)
and the pose-error statistics.  This runs once per experiment on 100 4x4 matrices, so
it stays plain torch on whatever device the poses live on; draws follow the
reference's order (angle, then axis, then translation, per pose) so that a CPU run
with the same seed reproduces the reference's CPU draws.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch


@dataclass
class NoiseConfig:
    """Reference noise.py:19-62."""

    rotation_noise_deg: float = 0.0
    translation_noise: float = 0.0
    translation_noise_pct: float = 0.0
    seed: Optional[int] = None

    def __str__(self) -> str:
        parts = []
        if self.rotation_noise_deg > 0:
            parts.append(f"rot{self.rotation_noise_deg:.1f}deg")
        if self.translation_noise_pct > 0:
            parts.append(f"trans{self.translation_noise_pct:.1f}pct")
        elif self.translation_noise > 0:
            parts.append(f"trans{self.translation_noise:.3f}")
        return "_".join(parts) if parts else "clean"

    @property
    def has_noise(self) -> bool:
        return self.rotation_noise_deg > 0 or self.translation_noise > 0 or self.translation_noise_pct > 0

    def get_translation_std(self, camera_distance: float) -> float:
        if self.translation_noise_pct > 0:
            return camera_distance * (self.translation_noise_pct / 100.0)
        return self.translation_noise


def set_noise_seed(seed: int) -> None:
    """Reference noise.py:65-68."""
    torch.manual_seed(seed)
    np.random.seed(seed)


def random_rotation_matrix(std_deg: float, device="cpu") -> torch.Tensor:
    """Reference noise.py:71-113: angle ~ N(0, std), axis uniform on the sphere, Rodrigues."""
    if std_deg == 0:
        return torch.eye(3, device=device)
    std_rad = std_deg * np.pi / 180.0
    angle = torch.randn(1, device=device) * std_rad
    axis = torch.randn(3, device=device)
    axis = axis / torch.norm(axis)
    K = torch.tensor([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]], device=device)
    return torch.eye(3, device=device) + torch.sin(angle) * K + (1 - torch.cos(angle)) * (K @ K)


def random_translation(std: float, device="cpu") -> torch.Tensor:
    """Reference noise.py:116-135."""
    if std == 0:
        return torch.zeros(3, device=device)
    return torch.randn(3, device=device) * std


def add_noise_to_pose(pose: torch.Tensor, rotation_noise_deg: float = 0.0,
                      translation_noise: float = 0.0) -> Tuple[torch.Tensor, dict]:
    """Reference noise.py:138-187: R_noisy = R_noise @ R, t_noisy = t + t_noise."""
    device = pose.device
    noisy = pose.clone()
    info = {"rotation_noise_deg": rotation_noise_deg, "translation_noise": translation_noise}
    if rotation_noise_deg > 0:
        R_noise = random_rotation_matrix(rotation_noise_deg, device)
        noisy[:3, :3] = R_noise @ pose[:3, :3]
        angle = torch.acos(torch.clamp((torch.trace(R_noise) - 1) / 2, -1, 1))
        info["actual_rotation_deg"] = float(angle * 180 / np.pi)
    if translation_noise > 0:
        t_noise = random_translation(translation_noise, device)
        noisy[:3, 3] = pose[:3, 3] + t_noise
        info["actual_translation_norm"] = float(torch.norm(t_noise))
    return noisy, info


def add_noise_to_poses(poses: torch.Tensor, noise_config: NoiseConfig) -> Tuple[torch.Tensor, list]:
    """Reference noise.py:190-234 (translation std relative to each camera's distance)."""
    if noise_config.seed is not None:
        set_noise_seed(noise_config.seed)
    out, infos = [], []
    for i in range(poses.shape[0]):
        dist = torch.norm(poses[i][:3, 3]).item()
        p, info = add_noise_to_pose(poses[i], rotation_noise_deg=noise_config.rotation_noise_deg,
                                    translation_noise=noise_config.get_translation_std(dist))
        out.append(p)
        infos.append(info)
    return torch.stack(out, dim=0), infos


def compute_pose_error(pose_gt: torch.Tensor, pose_noisy: torch.Tensor) -> dict:
    """Reference noise.py:237-268: geodesic rotation angle of R_gt^T R and translation distance."""
    R_diff = pose_gt[:3, :3].T @ pose_noisy[:3, :3]
    cos = torch.clamp((torch.trace(R_diff) - 1) / 2, -1.0, 1.0)
    rot_deg = float(torch.acos(cos) * 180 / np.pi)
    trans = float(torch.norm(pose_gt[:3, 3] - pose_noisy[:3, 3]))
    return {"rotation_error_deg": rot_deg, "translation_error": trans}
