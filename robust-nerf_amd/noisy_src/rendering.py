"""
Volume rendering — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src/rendering.py``.

``raw2outputs`` is the HIP alpha-composite (csrc/composite.hip); ``render_rays``
chains the HIP stages coarse sampling -> fused MLP -> composite -> inverse-CDF
sampling -> fused MLP -> composite exactly as rendering.py:119-240 does, and
``NeRFRenderer`` keeps the reference's chunking.
"""

from __future__ import annotations

from typing import Callable, Dict, Optional

import torch
import torch.nn as nn

from . import ops
from .config import RenderConfig
from .model import NeRF


def raw2outputs(rgb: torch.Tensor, sigma: torch.Tensor, z_vals: torch.Tensor, rays_d: torch.Tensor,
                raw_noise_std: float = 0.0, white_background: bool = True,
                noise: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """Reference rendering.py:20-116.  ``noise`` replaces randn_like(sigma)*std (:79)."""
    lead = z_vals.shape[:-1]
    S = z_vals.shape[-1]
    if raw_noise_std > 0.0 and noise is None:
        noise = torch.randn(*lead, S, device=z_vals.device) * raw_noise_std
    if raw_noise_std <= 0.0:
        noise = None
    rgb_map, depth, acc, weights = ops.composite(
        rgb.reshape(-1, S, 3), sigma.reshape(-1, S), z_vals.reshape(-1, S), rays_d.reshape(-1, 3),
        noise=None if noise is None else noise.reshape(-1, S), white_background=white_background)
    return {
        "rgb_map": rgb_map.reshape(*lead, 3),
        "depth_map": depth.reshape(lead),
        "acc_map": acc.reshape(lead),
        "weights": weights.reshape(*lead, S),
    }


def _outputs(rgb, sigma, z_vals, rays_d, raw_noise_std, white_background, target_rgb, loss_scale, net=None):
    """raw2outputs, or with a target its training form fused with the MSE loss (one
    launch, summing the loss with ``net``'s ticket; the dict then also holds "loss")."""
    if target_rgb is None:
        return raw2outputs(rgb, sigma, z_vals, rays_d, raw_noise_std=raw_noise_std,
                           white_background=white_background)
    S = z_vals.shape[-1]
    noise = None
    if raw_noise_std > 0.0:
        noise = torch.randn(*z_vals.shape[:-1], S, device=z_vals.device) * raw_noise_std
    loss, rgb_map, depth, acc, weights = ops.composite_mse(
        rgb.reshape(-1, S, 3), sigma.reshape(-1, S), z_vals.reshape(-1, S), rays_d.reshape(-1, 3), target_rgb,
        noise=None if noise is None else noise.reshape(-1, S), white_background=white_background,
        grad_scale=loss_scale,
        ticket=net.loss_ticket(z_vals.device) if hasattr(net, "loss_ticket") else None)
    return {"rgb_map": rgb_map, "depth_map": depth, "acc_map": acc, "weights": weights, "loss": loss}


def render_rays(model_coarse: NeRF, model_fine: Optional[NeRF], rays_o: torch.Tensor, rays_d: torch.Tensor,
                config: RenderConfig, is_train: bool = True, t_rand: Optional[torch.Tensor] = None,
                u: Optional[torch.Tensor] = None, return_aux: bool = False,
                coarse_stream: Optional[torch.cuda.Stream] = None,
                coarse_backward: Optional[Callable[[Dict[str, torch.Tensor]], None]] = None,
                target_rgb: Optional[torch.Tensor] = None, loss_scale: float = 1.0
                ) -> Dict[str, torch.Tensor]:
    """Reference rendering.py:119-240.  ``t_rand`` / ``u`` inject the jitter and
    inverse-CDF uniforms (otherwise drawn with torch.rand as the reference does).

    ``coarse_stream``: the coarse network's forward and compositing run on that stream
    (forked from and joined back into the current one), so autograd runs their backward
    there too, beside the fine network's (the two chains are independent: the fine
    samples depend on the coarse weights only through detached z values, reference
    rays.py:325).  Same kernels, same results; the caller joins the stream after
    ``backward``.  ``coarse_backward(out_c)``, with a coarse stream: called on that stream
    right after the coarse compositing (the caller runs the coarse loss's backward there),
    and the current stream waits only for the coarse FORWARD, so the coarse backward runs
    beside the fine sampling and forward.

    ``target_rgb`` (B,3), training: the MSE losses of train.py:89/98 are computed with the
    compositing (ops.composite_mse: one pass that also prepares the backward) and returned
    as "loss_coarse" / "loss_fine"; their gradients carry ``loss_scale``."""
    perturb = config.perturb if is_train else False
    raw_noise_std = config.raw_noise_std if is_train else 0.0
    N_rays = rays_o.shape[0]
    Nc = config.num_samples
    if perturb and t_rand is None:
        t_rand = torch.rand(N_rays, Nc, device=rays_o.device)
    # the view directions per sample (rendering.py:165) come out of the sampling launch
    pts, z_c, vd = ops.stratified_sample(rays_o, rays_d, config.near, config.far, Nc,
                                         t_rand=t_rand if perturb else None, viewdirs=True)
    if coarse_stream is not None:
        main = torch.cuda.current_stream(rays_o.device)
        coarse_stream.wait_stream(main)
        # these blocks come from the current stream's pool and the coarse chain (its
        # backward included, which may still run after this function returns) reads
        # them on the coarse stream: without the record the allocator could hand them
        # to the fine chain's allocations while the coarse kernels still read them
        for t in (pts, vd, z_c, rays_d) + ((target_rgb,) if target_rgb is not None else ()):
            t.record_stream(coarse_stream)
        with torch.cuda.stream(coarse_stream):
            rgb_c, sigma_c = model_coarse(pts.reshape(-1, 3), vd)
            out_c = _outputs(rgb_c.reshape(N_rays, Nc, 3), sigma_c.reshape(N_rays, Nc, 1), z_c, rays_d,
                             raw_noise_std, config.white_background, target_rgb, loss_scale, model_coarse)
            if coarse_backward is not None:
                forward_done = coarse_stream.record_event()
                coarse_backward(out_c)
        if coarse_backward is not None:
            main.wait_event(forward_done)
        else:
            main.wait_stream(coarse_stream)
    else:
        rgb_c, sigma_c = model_coarse(pts.reshape(-1, 3), vd)
        out_c = _outputs(rgb_c.reshape(N_rays, Nc, 3), sigma_c.reshape(N_rays, Nc, 1), z_c, rays_d,
                         raw_noise_std, config.white_background, target_rgb, loss_scale, model_coarse)
    results = {
        "rgb_coarse": out_c["rgb_map"],
        "depth_coarse": out_c["depth_map"],
        "acc_coarse": out_c["acc_map"],
    }
    if "loss" in out_c:
        results["loss_coarse"] = out_c["loss"]
    aux = {"z_coarse": z_c, "weights_coarse": out_c["weights"]}
    if config.use_hierarchical and model_fine is not None:
        Nf = config.num_samples_fine
        det = not is_train
        if not det and u is None:
            u = torch.rand(N_rays, Nf, device=rays_o.device)
        pts_f, z_f, vd_f = ops.sample_hierarchical(rays_o, rays_d, z_c, out_c["weights"], Nf, u=None if det else u,
                                                   viewdirs=True)
        T = z_f.shape[-1]
        rgb_f, sigma_f = model_fine(pts_f.reshape(-1, 3), vd_f)
        out_f = _outputs(rgb_f.reshape(N_rays, T, 3), sigma_f.reshape(N_rays, T, 1), z_f, rays_d,
                         raw_noise_std, config.white_background, target_rgb, loss_scale, model_fine)
        if "loss" in out_f:
            results["loss_fine"] = out_f["loss"]
        results["rgb_fine"] = out_f["rgb_map"]
        results["depth_fine"] = out_f["depth_map"]
        results["acc_fine"] = out_f["acc_map"]
        aux["z_fine"] = z_f
        aux["weights_fine"] = out_f["weights"]
    if return_aux:
        return results, aux
    return results


class NeRFRenderer(nn.Module):
    """Reference rendering.py:243-323 (chunked rendering; owns both networks)."""

    def __init__(self, model_coarse: NeRF, model_fine: Optional[NeRF], config: RenderConfig):
        super().__init__()
        self.model_coarse = model_coarse
        self.model_fine = model_fine
        self.config = config

    def forward(self, rays_o: torch.Tensor, rays_d: torch.Tensor, chunk_size: int = 1024 * 32,
                is_train: bool = True) -> Dict[str, torch.Tensor]:
        N_rays = rays_o.shape[0]
        if N_rays <= chunk_size:
            return render_rays(self.model_coarse, self.model_fine, rays_o, rays_d, self.config, is_train=is_train)
        all_results: Dict[str, list] = {}
        for i in range(0, N_rays, chunk_size):
            chunk = render_rays(self.model_coarse, self.model_fine, rays_o[i:i + chunk_size],
                                rays_d[i:i + chunk_size], self.config, is_train=is_train)
            for k, v in chunk.items():
                all_results.setdefault(k, []).append(v)
        return {k: torch.cat(v, dim=0) for k, v in all_results.items()}
