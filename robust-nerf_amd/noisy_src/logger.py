"""
Experiment logging — the reference's metric containers, CSV schema and output layout
(ShawnnnLiu/Robust-NeRF ``noisy_src/logger.py:26-368``), so output folders stay
comparable with the reference's ``outputs/<exp>/``: ``config.json``, ``summary.json``,
``logs/train_metrics.csv`` (one row per iteration, flushed), ``logs/val_metrics.csv``,
``images/{tag}_{pred,gt,comparison,depth}_{iteration:07d}.png``.  TensorBoard is optional
in the reference and not installed here, so that backend reports itself unavailable.
"""

from __future__ import annotations

import csv
import json
import time
from dataclasses import asdict, dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional

import numpy as np
import torch


@dataclass
class TrainingMetrics:
    """Reference logger.py:26-39 (column order of train_metrics.csv)."""

    iteration: int
    loss: float
    loss_coarse: float
    loss_fine: Optional[float] = None
    psnr: float = 0.0
    learning_rate: float = 0.0
    time_per_iter: float = 0.0
    rays_per_sec: float = 0.0

    def to_dict(self) -> Dict[str, Any]:
        return {k: v for k, v in asdict(self).items() if v is not None}


@dataclass
class ValidationMetrics:
    """Reference logger.py:42-57."""

    iteration: int
    psnr: float
    ssim: float = 0.0
    lpips: Optional[float] = None
    mse: float = 0.0
    per_image_psnr: List[float] = field(default_factory=list)
    per_image_ssim: List[float] = field(default_factory=list)

    def to_dict(self) -> Dict[str, Any]:
        return {k: v for k, v in asdict(self).items() if v is not None and v != []}


class TensorBoardLogger:
    """Reference logger.py:60-108.  ``tensorboard`` is not installed in this image, so
    ``available`` is False and every call is a no-op, as in the reference without it."""

    def __init__(self, log_dir: Path):
        self.writer = None
        try:  # pragma: no cover - optional dependency
            from torch.utils.tensorboard import SummaryWriter
            self.writer = SummaryWriter(str(log_dir))
        except Exception:
            self.writer = None
        self.available = self.writer is not None

    def log_scalar(self, tag: str, value: float, step: int) -> None:
        if self.available:
            self.writer.add_scalar(tag, value, step)

    def close(self) -> None:
        if self.writer is not None:
            self.writer.close()


class CSVLogger:
    """Reference logger.py:111-156: header from the first row's keys, flushed per row."""

    def __init__(self, log_dir: Path):
        self.log_dir = Path(log_dir)
        self.log_dir.mkdir(parents=True, exist_ok=True)
        self.train_file = self.log_dir / "train_metrics.csv"
        self.val_file = self.log_dir / "val_metrics.csv"
        self._w = {}

    def _row(self, key: str, path: Path, data: Dict[str, Any]) -> None:
        if key not in self._w:
            fh = open(path, "w", newline="")
            w = csv.DictWriter(fh, fieldnames=list(data.keys()))
            w.writeheader()
            self._w[key] = (fh, w)
        fh, w = self._w[key]
        w.writerow(data)
        fh.flush()

    def log_train(self, metrics: TrainingMetrics) -> None:
        self._row("train", self.train_file, metrics.to_dict())

    def log_val(self, metrics: ValidationMetrics) -> None:
        self._row("val", self.val_file, {k: v for k, v in metrics.to_dict().items() if not isinstance(v, list)})

    def close(self) -> None:
        for fh, _ in self._w.values():
            fh.close()
        self._w.clear()


def _save_png(img: torch.Tensor, path: Path) -> None:
    from PIL import Image
    arr = (img.detach().float().cpu().numpy() * 255).clip(0, 255).astype(np.uint8)
    Image.fromarray(arr).save(path)


def depth_to_colormap(depth: torch.Tensor) -> torch.Tensor:
    """Reference logger.py:290-302: min-max normalised depth through a turbo-like ramp."""
    depth = depth.detach().float().cpu()
    n = (depth - depth.min()) / (depth.max() - depth.min() + 1e-8)
    return torch.stack([torch.clamp(4 * n - 1.5, 0, 1), torch.clamp(2 - 4 * torch.abs(n - 0.5), 0, 1),
                        torch.clamp(1.5 - 4 * n, 0, 1)], dim=-1)


class ExperimentLogger:
    """Reference logger.py:159-368: CSVs under ``logs/``, PNGs under ``images/``,
    ``config.json`` and a ``summary.json`` of run metadata and final/best metrics."""

    def __init__(self, output_dir: Path, experiment_name: str = "experiment", use_tensorboard: bool = True):
        self.output_dir = Path(output_dir)
        self.experiment_name = experiment_name
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.logs_dir = self.output_dir / "logs"
        self.images_dir = self.output_dir / "images"
        self.logs_dir.mkdir(exist_ok=True)
        self.images_dir.mkdir(exist_ok=True)
        self.csv_logger = CSVLogger(self.logs_dir)
        self.tb_logger = TensorBoardLogger(self.logs_dir / "tensorboard") if use_tensorboard else None
        self.train_history: List[TrainingMetrics] = []
        self.val_history: List[ValidationMetrics] = []
        self.start_time = time.time()
        self.metadata: Dict[str, Any] = {"experiment_name": experiment_name, "start_time": datetime.now().isoformat(),
                                         "output_dir": str(output_dir)}

    def log_training(self, metrics: TrainingMetrics) -> None:
        self.train_history.append(metrics)
        self.csv_logger.log_train(metrics)
        if self.tb_logger is not None and self.tb_logger.available:
            for k in ("loss", "loss_coarse", "loss_fine", "psnr", "learning_rate", "rays_per_sec"):
                v = getattr(metrics, k)
                if v is not None:
                    self.tb_logger.log_scalar(f"train/{k}", v, metrics.iteration)

    def log_validation(self, metrics: ValidationMetrics) -> None:
        self.val_history.append(metrics)
        self.csv_logger.log_val(metrics)
        if self.tb_logger is not None and self.tb_logger.available:
            for k in ("psnr", "ssim", "mse", "lpips"):
                v = getattr(metrics, k)
                if v is not None:
                    self.tb_logger.log_scalar(f"val/{k}", v, metrics.iteration)

    def log_images(self, tag: str, pred: torch.Tensor, gt: torch.Tensor, iteration: int,
                   depth: Optional[torch.Tensor] = None) -> None:
        """Reference logger.py:242-281 (pred, gt, side-by-side comparison, depth)."""
        _save_png(pred, self.images_dir / f"{tag}_pred_{iteration:07d}.png")
        _save_png(gt, self.images_dir / f"{tag}_gt_{iteration:07d}.png")
        _save_png(torch.cat([gt.detach().float().cpu(), pred.detach().float().cpu()], dim=1),
                  self.images_dir / f"{tag}_comparison_{iteration:07d}.png")
        if depth is not None:
            _save_png(depth_to_colormap(depth), self.images_dir / f"{tag}_depth_{iteration:07d}.png")

    def log_model_info(self, model: torch.nn.Module, name: str = "model") -> None:
        """Reference logger.py:304-313."""
        total = sum(p.numel() for p in model.parameters())
        trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
        self.metadata[f"{name}_total_params"] = total
        self.metadata[f"{name}_trainable_params"] = trainable
        print(f"{name}: {total:,} total params, {trainable:,} trainable")

    def log_config(self, config: Any) -> None:
        cfg = self._config_to_dict(config) if hasattr(config, "__dict__") else config
        self.metadata["config"] = cfg
        (self.output_dir / "config.json").write_text(json.dumps(cfg, indent=2, default=str))

    def _config_to_dict(self, obj: Any) -> Any:
        if hasattr(obj, "__dataclass_fields__"):
            return {k: self._config_to_dict(v) for k, v in obj.__dict__.items()}
        if isinstance(obj, Path):
            return str(obj)
        if isinstance(obj, (list, tuple)):
            return [self._config_to_dict(v) for v in obj]
        return obj

    def save_summary(self) -> None:
        """Reference logger.py:338-363."""
        self.metadata["end_time"] = datetime.now().isoformat()
        self.metadata["total_time_seconds"] = time.time() - self.start_time
        self.metadata["total_iterations"] = len(self.train_history)
        if self.val_history:
            final = self.val_history[-1]
            self.metadata["final_val_psnr"] = final.psnr
            self.metadata["final_val_ssim"] = final.ssim
            if final.lpips:
                self.metadata["final_val_lpips"] = final.lpips
            self.metadata["best_val_psnr"] = max(v.psnr for v in self.val_history)
            self.metadata["best_val_ssim"] = max(v.ssim for v in self.val_history)
        (self.output_dir / "summary.json").write_text(json.dumps(self.metadata, indent=2, default=str))

    def close(self) -> None:
        self.csv_logger.close()
        if self.tb_logger is not None:
            self.tb_logger.close()
