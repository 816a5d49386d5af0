"""
Experiment logging — the reference's metric containers and CSV schema
(ShawnnnLiu/Robust-NeRF ``noisy_src/logger.py:26-156``), so output folders stay
comparable with the reference's ``outputs/*/train_metrics.csv`` / ``val_metrics.csv``.
TensorBoard is optional in the reference and not installed here; ``ExperimentLogger``
writes the CSVs, the config/summary JSON and PNG previews.
"""

from __future__ import annotations

import csv
import json
from dataclasses import asdict, dataclass, field, is_dataclass
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


class ExperimentLogger:
    """Reference logger.py:159-368 (CSV + JSON + PNG parts)."""

    def __init__(self, output_dir: Path, experiment_name: str, use_tensorboard: bool = False):
        self.output_dir = Path(output_dir)
        self.experiment_name = experiment_name
        self.output_dir.mkdir(parents=True, exist_ok=True)
        (self.output_dir / "images").mkdir(exist_ok=True)
        self.csv = CSVLogger(self.output_dir)
        self.train_history: List[Dict[str, Any]] = []
        self.val_history: List[Dict[str, Any]] = []

    def log_training(self, metrics: TrainingMetrics) -> None:
        self.csv.log_train(metrics)
        self.train_history.append(metrics.to_dict())

    def log_validation(self, metrics: ValidationMetrics) -> None:
        self.csv.log_val(metrics)
        self.val_history.append(metrics.to_dict())

    def log_images(self, tag: str, pred: torch.Tensor, gt: Optional[torch.Tensor] = None, iteration: int = 0,
                   depth: Optional[torch.Tensor] = None) -> None:
        self._save_image(pred, self.output_dir / "images" / f"{tag}_pred_{iteration:06d}.png")
        if gt is not None:
            self._save_image(gt, self.output_dir / "images" / f"{tag}_gt_{iteration:06d}.png")

    def _save_image(self, img: torch.Tensor, path: Path) -> None:
        from PIL import Image
        arr = (img.detach().float().clamp(0, 1).cpu().numpy() * 255).astype(np.uint8)
        Image.fromarray(arr).save(path)

    def log_config(self, config: Any) -> None:
        (self.output_dir / "config.json").write_text(json.dumps(self._config_to_dict(config), indent=2, default=str))

    def _config_to_dict(self, obj: Any) -> Any:
        if is_dataclass(obj):
            return {k: self._config_to_dict(v) for k, v in asdict(obj).items()}
        return obj

    def save_summary(self) -> None:
        summary = {"experiment_name": self.experiment_name, "total_iterations": len(self.train_history)}
        if self.val_history:
            best = max(self.val_history, key=lambda m: m.get("psnr", float("-inf")))
            summary["best_psnr"] = best.get("psnr")
            summary["final_psnr"] = self.val_history[-1].get("psnr")
        (self.output_dir / "summary.json").write_text(json.dumps(summary, indent=2))

    def close(self) -> None:
        self.save_summary()
        self.csv.close()
