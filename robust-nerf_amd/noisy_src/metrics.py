"""
Image-quality metrics — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src/metrics.py``.

Evaluation-side, not the training hot path: PSNR / MSE / SSIM run
as device tensor ops on the rendered image where it lies (no host round trip).
LPIPS needs the ``lpips`` package and VGG weights from the network (metrics.py:119-168);
neither exists offline, so ``LPIPSMetric`` reports itself unavailable and returns
None, which ``compute_all_metrics`` skips exactly as the reference does.
"""

from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F


def compute_psnr(pred: torch.Tensor, target: torch.Tensor, max_val: float = 1.0) -> torch.Tensor:
    """Reference metrics.py:15-40: 20 log10(max) - 10 log10(mean((pred - target)^2))."""
    mse = torch.mean((pred - target) ** 2)
    if mse == 0:
        return torch.tensor(float("inf"))
    return 20.0 * torch.log10(torch.tensor(max_val)) - 10.0 * torch.log10(mse)


def compute_mse(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Reference metrics.py:43-45."""
    return torch.mean((pred - target) ** 2)


def _gaussian_window(size: int, sigma: float = 1.5) -> torch.Tensor:
    coords = torch.arange(size, dtype=torch.float32) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    g = g / g.sum()
    return g.outer(g)


def compute_ssim(pred: torch.Tensor, target: torch.Tensor, window_size: int = 11, C1: float = 0.01 ** 2,
                 C2: float = 0.03 ** 2) -> torch.Tensor:
    """Reference metrics.py:48-116: mean SSIM with an 11x11 Gaussian window (sigma 1.5),
    zero padding, per-channel (grouped) convolutions."""
    pred = pred.float()
    target = target.float()
    if pred.dim() == 3:
        pred = pred.permute(2, 0, 1).unsqueeze(0)
        target = target.permute(2, 0, 1).unsqueeze(0)
    elif pred.dim() == 2:
        pred = pred.unsqueeze(0).unsqueeze(0)
        target = target.unsqueeze(0).unsqueeze(0)
    C = pred.shape[1]
    window = _gaussian_window(window_size).to(pred.device)[None, None].expand(C, 1, window_size, window_size)
    pad = window_size // 2

    def blur(x):
        return F.conv2d(x, window, padding=pad, groups=C)

    mu_p, mu_t = blur(pred), blur(target)
    mu_p2, mu_t2, mu_pt = mu_p ** 2, mu_t ** 2, mu_p * mu_t
    s_p = blur(pred ** 2) - mu_p2
    s_t = blur(target ** 2) - mu_t2
    s_pt = blur(pred * target) - mu_pt
    ssim_map = ((2 * mu_pt + C1) * (2 * s_pt + C2)) / ((mu_p2 + mu_t2 + C1) * (s_p + s_t + C2))
    return ssim_map.mean()


class LPIPSMetric:
    """Reference metrics.py:119-168.  The ``lpips`` package and its VGG weights are not
    available offline: ``available`` is False and calls return None."""

    def __init__(self, net: str = "vgg", device: str = "cuda"):
        self.net = net
        self.device = device
        try:  # pragma: no cover - not installed in this image
            import lpips  # noqa: F401
            self.available = False  # weights would need a download; never fetched here
        except ImportError:
            self.available = False

    def __call__(self, pred: torch.Tensor, target: torch.Tensor) -> Optional[torch.Tensor]:
        return None


def compute_all_metrics(pred: torch.Tensor, target: torch.Tensor,
                        lpips_metric: Optional[LPIPSMetric] = None) -> Dict[str, float]:
    """Reference metrics.py:171-205."""
    metrics = {
        "mse": compute_mse(pred, target).item(),
        "psnr": compute_psnr(pred, target).item(),
        "ssim": compute_ssim(pred, target).item(),
    }
    if lpips_metric is not None:
        v = lpips_metric(pred, target)
        if v is not None:
            metrics["lpips"] = v.item()
    return metrics
