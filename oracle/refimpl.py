"""ORACLE — test infrastructure only; never shipped, never on the product path.

CPU restatement (PyTorch on ``device="cpu"``) of the reference hot path of
ShawnnnLiu/Robust-NeRF, op for op, with every random draw injectable so the HIP
path can be compared on identical inputs.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import it.

Parity status: PARTIALLY PINNED.  The reference could not be imported or run in
this container (the denial is recorded in SURVEY.md §8c), and its own tests
(`noisy_src/test_baseline.py`) pin only shapes and ranges.  This restatement is
pinned by (a) the reference's run artifacts read as raw bytes — the dead
rotation gradient of CameraPoseParameters in every ``outputs/*/final_poses.pt``
(R_opt == R_init bit for bit, t moved), the LambdaLR value logged at iteration 0
in ``outputs/*/logs/train_metrics.csv`` and the parameter count 595,844 of
every ``summary.json`` — see tests/golden/ and tests/test_oracle.py; and (b)
analytic known-answer tests.  Everything else rests on the
line-by-line restatement below (file:line cited per function).
"""

from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# rays.py
# --------------------------------------------------------------------------
def get_ray_directions(H: int, W: int, focal: float, center=None) -> torch.Tensor:
    """Reference noisy_src/rays.py:17-64 (meshgrid 'xy', no pixel-centre offset)."""
    if center is None:
        cx, cy = W / 2.0, H / 2.0
    else:
        cx, cy = center
    i, j = torch.meshgrid(
        torch.arange(W, dtype=torch.float32),
        torch.arange(H, dtype=torch.float32),
        indexing="xy",
    )
    return torch.stack([(i - cx) / focal, -(j - cy) / focal, -torch.ones_like(i)], dim=-1)


def get_rays(directions: torch.Tensor, c2w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference noisy_src/rays.py:67-99."""
    rays_d = torch.sum(directions[..., None, :] * c2w[:3, :3], dim=-1)
    rays_d = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    rays_o = c2w[:3, 3].expand(rays_d.shape)
    return rays_o, rays_d


def sample_along_rays(rays_o, rays_d, near, far, num_samples, perturb=True, lindisp=False,
                      t_rand: Optional[torch.Tensor] = None):
    """Reference noisy_src/rays.py:145-210; ``t_rand`` replaces torch.rand at :204."""
    device = rays_o.device
    batch_shape = rays_o.shape[:-1]
    t_vals = torch.linspace(0.0, 1.0, num_samples, device=device)
    if lindisp:
        z_vals = 1.0 / (1.0 / near * (1.0 - t_vals) + 1.0 / far * t_vals)
    else:
        z_vals = near * (1.0 - t_vals) + far * t_vals
    z_vals = z_vals.expand(*batch_shape, num_samples)
    if perturb:
        mids = 0.5 * (z_vals[..., 1:] + z_vals[..., :-1])
        upper = torch.cat([mids, z_vals[..., -1:]], dim=-1)
        lower = torch.cat([z_vals[..., :1], mids], dim=-1)
        if t_rand is None:
            t_rand = torch.rand(*batch_shape, num_samples, device=device)
        z_vals = lower + (upper - lower) * t_rand
    pts = rays_o[..., None, :] + rays_d[..., None, :] * z_vals[..., :, None]
    return pts, z_vals


def sample_pdf(bins, weights, num_samples, det=False, u: Optional[torch.Tensor] = None):
    """Reference noisy_src/rays.py:213-279; ``u`` replaces torch.rand at :255."""
    device = weights.device
    weights = weights + 1e-5
    pdf = weights / torch.sum(weights, dim=-1, keepdim=True)
    cdf = torch.cumsum(pdf, dim=-1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], dim=-1)
    if det:
        u = torch.linspace(0.0, 1.0, num_samples, device=device)
        u = u.expand(*cdf.shape[:-1], num_samples)
    elif u is None:
        u = torch.rand(*cdf.shape[:-1], num_samples, device=device)
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.clamp(inds - 1, min=0)
    above = torch.clamp(inds, max=cdf.shape[-1] - 1)
    inds_g = torch.stack([below, above], dim=-1)
    cdf_g = torch.gather(cdf, -1, inds_g.reshape(*cdf.shape[:-1], -1)).reshape(*inds_g.shape)
    bins_g = torch.gather(bins, -1, inds_g.reshape(*bins.shape[:-1], -1)).reshape(*inds_g.shape)
    denom = cdf_g[..., 1] - cdf_g[..., 0]
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_g[..., 0]) / denom
    return bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0])


def sample_hierarchical(rays_o, rays_d, z_vals, weights, num_samples_fine, det=False,
                        u: Optional[torch.Tensor] = None):
    """Reference noisy_src/rays.py:282-333."""
    z_vals_mid = 0.5 * (z_vals[..., 1:] + z_vals[..., :-1])
    z_samples = sample_pdf(z_vals_mid, weights[..., 1:-1], num_samples_fine, det=det, u=u)
    z_samples = z_samples.detach()
    z_vals_fine, _ = torch.sort(torch.cat([z_vals, z_samples], dim=-1), dim=-1)
    pts_fine = rays_o[..., None, :] + rays_d[..., None, :] * z_vals_fine[..., :, None]
    return pts_fine, z_vals_fine


# --------------------------------------------------------------------------
# model.py
# --------------------------------------------------------------------------
class PositionalEncoding(nn.Module):
    """Reference noisy_src/model.py:20-80 (no pi factor; [x, sin f0x, cos f0x, ...])."""

    def __init__(self, num_freqs: int, include_input: bool = True, log_sampling: bool = True):
        super().__init__()
        self.num_freqs = num_freqs
        self.include_input = include_input
        if log_sampling:
            freq_bands = 2.0 ** torch.linspace(0.0, num_freqs - 1, num_freqs)
        else:
            freq_bands = torch.linspace(1.0, 2.0 ** (num_freqs - 1), num_freqs)
        self.register_buffer("freq_bands", freq_bands)

    @property
    def output_dim(self) -> int:
        return 2 * self.num_freqs + (1 if self.include_input else 0)

    def forward(self, x):
        out = [x] if self.include_input else []
        for freq in self.freq_bands:
            out.append(torch.sin(freq * x))
            out.append(torch.cos(freq * x))
        return torch.cat(out, dim=-1)


class NeRF(nn.Module):
    """Reference noisy_src/model.py:83-196 (same parameter names and order)."""

    def __init__(self, config=None):
        super().__init__()
        if config is None:
            from types import SimpleNamespace
            config = SimpleNamespace(pos_freqs=10, dir_freqs=4, hidden_dim=256,
                                     num_hidden_layers=8, skips=(4,), use_view_dirs=True)
        self.config = config
        self.pos_encoder = PositionalEncoding(config.pos_freqs, include_input=True)
        self.dir_encoder = PositionalEncoding(config.dir_freqs, include_input=True)
        pos_dim = 3 * self.pos_encoder.output_dim
        dir_dim = 3 * self.dir_encoder.output_dim
        self.pts_linears = nn.ModuleList()
        in_dim = pos_dim
        for i in range(config.num_hidden_layers):
            self.pts_linears.append(nn.Linear(in_dim, config.hidden_dim))
            in_dim = config.hidden_dim
            if i in config.skips:
                in_dim += pos_dim
        self.sigma_linear = nn.Linear(config.hidden_dim, 1)
        self.feature_linear = nn.Linear(config.hidden_dim, config.hidden_dim)
        if config.use_view_dirs:
            self.dir_linear = nn.Linear(config.hidden_dim + dir_dim, config.hidden_dim // 2)
        else:
            self.dir_linear = nn.Linear(config.hidden_dim, config.hidden_dim // 2)
        self.rgb_linear = nn.Linear(config.hidden_dim // 2, 3)

    def forward(self, x, d=None):
        x_enc = self.pos_encoder(x)
        h = x_enc
        for i, layer in enumerate(self.pts_linears):
            h = F.relu(layer(h))
            if i in self.config.skips:
                h = torch.cat([x_enc, h], dim=-1)
        sigma = F.relu(self.sigma_linear(h))
        feats = self.feature_linear(h)
        if self.config.use_view_dirs and d is not None:
            h_color = torch.cat([feats, self.dir_encoder(d)], dim=-1)
        else:
            h_color = feats
        h_color = F.relu(self.dir_linear(h_color))
        rgb = torch.sigmoid(self.rgb_linear(h_color))
        return rgb, sigma


def create_nerf(config=None):
    """Reference noisy_src/model.py:199-221."""
    return NeRF(config), NeRF(config)


# --------------------------------------------------------------------------
# rendering.py
# --------------------------------------------------------------------------
def raw2outputs(rgb, sigma, z_vals, rays_d, raw_noise_std=0.0, white_background=True,
                noise: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
    """Reference noisy_src/rendering.py:20-116; ``noise`` replaces randn_like at :79."""
    sigma = sigma.squeeze(-1)
    dists = z_vals[..., 1:] - z_vals[..., :-1]
    dists = torch.cat([dists, torch.full_like(dists[..., :1], 1e10)], dim=-1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    if raw_noise_std > 0.0:
        if noise is None:
            noise = torch.randn_like(sigma) * raw_noise_std
        sigma = sigma + noise
    alpha = 1.0 - torch.exp(-torch.relu(sigma) * dists)
    transmittance = torch.cumprod(
        torch.cat([torch.ones_like(alpha[..., :1]), 1.0 - alpha + 1e-10], dim=-1), dim=-1
    )[..., :-1]
    weights = alpha * transmittance
    rgb_map = torch.sum(weights[..., None] * rgb, dim=-2)
    depth_map = torch.sum(weights * z_vals, dim=-1)
    acc_map = torch.sum(weights, dim=-1)
    if white_background:
        rgb_map = rgb_map + (1.0 - acc_map[..., None])
    return {"rgb_map": rgb_map, "depth_map": depth_map, "acc_map": acc_map, "weights": weights}


def render_rays(model_coarse, model_fine, rays_o, rays_d, config, is_train=True,
                t_rand=None, u=None, noise_c=None, noise_f=None, return_aux=False):
    """Reference noisy_src/rendering.py:119-240 with injected randoms."""
    perturb = config.perturb if is_train else False
    raw_noise_std = config.raw_noise_std if is_train else 0.0
    viewdirs = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    pts_coarse, z_vals_coarse = sample_along_rays(
        rays_o, rays_d, config.near, config.far, config.num_samples, perturb=perturb, t_rand=t_rand)
    N_rays = rays_o.shape[0]
    Nc = config.num_samples
    pts_flat = pts_coarse.reshape(-1, 3)
    viewdirs_flat = viewdirs[:, None, :].expand(-1, Nc, -1).reshape(-1, 3)
    rgb_c, sigma_c = model_coarse(pts_flat, viewdirs_flat)
    out_c = raw2outputs(rgb_c.reshape(N_rays, Nc, 3), sigma_c.reshape(N_rays, Nc, 1), z_vals_coarse,
                        rays_d, raw_noise_std, config.white_background, noise=noise_c)
    results = {"rgb_coarse": out_c["rgb_map"], "depth_coarse": out_c["depth_map"],
               "acc_coarse": out_c["acc_map"]}
    aux = {"z_coarse": z_vals_coarse, "weights_coarse": out_c["weights"]}
    if config.use_hierarchical and model_fine is not None:
        pts_fine, z_vals_fine = sample_hierarchical(
            rays_o, rays_d, z_vals_coarse, out_c["weights"], config.num_samples_fine,
            det=not is_train, u=u)
        Nf = z_vals_fine.shape[-1]
        pts_flat = pts_fine.reshape(-1, 3)
        viewdirs_flat = viewdirs[:, None, :].expand(-1, Nf, -1).reshape(-1, 3)
        rgb_f, sigma_f = model_fine(pts_flat, viewdirs_flat)
        out_f = raw2outputs(rgb_f.reshape(N_rays, Nf, 3), sigma_f.reshape(N_rays, Nf, 1), z_vals_fine,
                            rays_d, raw_noise_std, config.white_background, noise=noise_f)
        results["rgb_fine"] = out_f["rgb_map"]
        results["depth_fine"] = out_f["depth_map"]
        results["acc_fine"] = out_f["acc_map"]
        aux["z_fine"] = z_vals_fine
        aux["weights_fine"] = out_f["weights"]
    if return_aux:
        return results, aux
    return results


# --------------------------------------------------------------------------
# train_pose_opt.py / data_pose_opt.py
# --------------------------------------------------------------------------
class CameraPoseParameters(nn.Module):
    """Reference noisy_src/train_pose_opt.py:53-226 (incl. the theta<1e-6 where rule)."""

    def __init__(self, initial_poses, learn_rotation=True, learn_translation=True):
        super().__init__()
        self.n_poses = initial_poses.shape[0]
        self.learn_rotation = learn_rotation
        self.learn_translation = learn_translation
        self.register_buffer("initial_poses", initial_poses.clone())
        z = torch.zeros(self.n_poses, 3, device=initial_poses.device)
        if learn_rotation:
            self.rotation_deltas = nn.Parameter(z.clone())
        else:
            self.register_buffer("rotation_deltas", z.clone())
        if learn_translation:
            self.translation_deltas = nn.Parameter(z.clone())
        else:
            self.register_buffer("translation_deltas", z.clone())

    def axis_angle_to_rotation_matrix(self, axis_angle):
        batch_shape = axis_angle.shape[:-1]
        axis_angle = axis_angle.reshape(-1, 3)
        angle = torch.norm(axis_angle, dim=-1, keepdim=True)
        small_angle = angle < 1e-6
        angle = torch.where(small_angle, torch.ones_like(angle), angle)
        axis = axis_angle / angle
        K = self._skew_symmetric(axis)
        K2 = torch.bmm(K, K)
        I = torch.eye(3, device=axis_angle.device).unsqueeze(0).expand(axis.shape[0], 3, 3)
        sin_angle = torch.sin(angle).unsqueeze(-1)
        cos_angle = torch.cos(angle).unsqueeze(-1)
        R = I + sin_angle * K + (1 - cos_angle) * K2
        R = torch.where(small_angle.reshape(-1, 1, 1), I, R)
        return R.reshape(*batch_shape, 3, 3)

    def _skew_symmetric(self, v):
        zeros = torch.zeros(v.shape[0], device=v.device)
        return torch.stack([
            torch.stack([zeros, -v[:, 2], v[:, 1]], dim=-1),
            torch.stack([v[:, 2], zeros, -v[:, 0]], dim=-1),
            torch.stack([-v[:, 1], v[:, 0], zeros], dim=-1),
        ], dim=1)

    def get_poses(self, indices=None):
        if indices is None:
            indices = torch.arange(self.n_poses, device=self.initial_poses.device)
        poses_init = self.initial_poses[indices]
        if self.learn_rotation:
            R_delta = self.axis_angle_to_rotation_matrix(self.rotation_deltas[indices])
            R_new = torch.bmm(R_delta, poses_init[:, :3, :3])
        else:
            R_new = poses_init[:, :3, :3]
        if self.learn_translation:
            t_new = poses_init[:, :3, 3] + self.translation_deltas[indices]
        else:
            t_new = poses_init[:, :3, 3]
        poses = torch.zeros_like(poses_init)
        poses[:, :3, :3] = R_new
        poses[:, :3, 3] = t_new
        poses[:, 3, 3] = 1.0
        return poses

    def get_all_poses(self):
        return self.get_poses()


def get_rays_from_pixels(image_indices, pixel_coords, poses, H, W, focal):
    """Reference noisy_src/data_pose_opt.py:83-148 + :200-223 (poses indexed by image)."""
    ray_directions = get_ray_directions(H, W, focal).to(pixel_coords.device, poses.dtype)
    batch_size = image_indices.shape[0]
    unique_img_indices = torch.unique(image_indices)
    selected = poses[unique_img_indices]
    # reference: torch.zeros(batch_size, 3) (fp32); the dtype follows the poses so the
    # same restatement can run in fp64 for error studies
    rays_o = torch.zeros(batch_size, 3, device=pixel_coords.device, dtype=poses.dtype)
    rays_d = torch.zeros(batch_size, 3, device=pixel_coords.device, dtype=poses.dtype)
    parts = []
    for k, img_idx in enumerate(unique_img_indices):
        mask = image_indices == img_idx
        pc = pixel_coords[mask]
        u = pc[:, 0].long()
        v = pc[:, 1].long()
        o, d = get_rays(ray_directions[v, u], selected[k])
        parts.append((mask, o, d))
    for mask, o, d in parts:
        rays_o[mask] = o
        rays_d[mask] = d
    return rays_o, rays_d


# --------------------------------------------------------------------------
# train.py / metrics.py
# --------------------------------------------------------------------------
def compute_psnr(pred, target, max_val: float = 1.0):
    """Reference noisy_src/metrics.py:15-40."""
    mse = torch.mean((pred - target) ** 2)
    if mse == 0:
        return torch.tensor(float("inf"))
    return 20.0 * torch.log10(torch.tensor(max_val)) - 10.0 * torch.log10(mse)


def lr_lambda(step: int, lr_decay: int = 250) -> float:
    """Reference noisy_src/train.py:405-411 (decay 0.1 every lr_decay*1000 steps)."""
    return 0.1 ** (step / (lr_decay * 1000))


class TrainState:
    """train.py:398-411 optimiser + scheduler around the two oracle networks."""

    def __init__(self, model_coarse, model_fine, lr=5e-4, lr_decay=250):
        params = list(model_coarse.parameters())
        if model_fine is not None:
            params += list(model_fine.parameters())
        self.params = params
        self.optimizer = torch.optim.Adam(params, lr=lr)
        self.scheduler = torch.optim.lr_scheduler.LambdaLR(
            self.optimizer, lambda s: lr_lambda(s, lr_decay))


def train_step(model_coarse, model_fine, state: TrainState, rays_o, rays_d, target_rgb, config,
               t_rand=None, u=None, max_norm=1.0):
    """Reference noisy_src/train.py:68-119 (+ scheduler.step at :461)."""
    state.optimizer.zero_grad()
    outputs = render_rays(model_coarse, model_fine, rays_o, rays_d, config, is_train=True,
                          t_rand=t_rand, u=u)
    loss_coarse = torch.mean((outputs["rgb_coarse"] - target_rgb) ** 2)
    loss = loss_coarse
    loss_fine = None
    if "rgb_fine" in outputs:
        loss_fine = torch.mean((outputs["rgb_fine"] - target_rgb) ** 2)
        loss = loss_coarse + loss_fine
    loss.backward()
    torch.nn.utils.clip_grad_norm_(state.params, max_norm=max_norm)
    state.optimizer.step()
    state.scheduler.step()
    return {"loss": float(loss.detach()), "loss_coarse": float(loss_coarse.detach()),
            "loss_fine": None if loss_fine is None else float(loss_fine.detach())}


def flat_params(model: nn.Module) -> torch.Tensor:
    """Parameters in nn.Module.parameters() order, flattened (the C-ABI layout)."""
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()])


def flat_grads(model: nn.Module) -> torch.Tensor:
    return torch.cat([
        (p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in model.parameters()
    ])


def num_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def mlp_flops_per_sample(pos_freqs=10, dir_freqs=4, hidden=256, n_layers=8, skips=(4,)) -> int:
    """Algorithmic MACs of one NeRF MLP evaluation (593,408)."""
    pos_dim = 3 * (1 + 2 * pos_freqs)
    dir_dim = 3 * (1 + 2 * dir_freqs)
    macs = 0
    in_dim = pos_dim
    for i in range(n_layers):
        macs += in_dim * hidden
        in_dim = hidden + (pos_dim if i in skips else 0)
    macs += in_dim * 1 + in_dim * hidden + (hidden + dir_dim) * (hidden // 2) + (hidden // 2) * 3
    return macs


def compute_pose_error(pose_gt, pose_noisy):
    """Reference noisy_src/noise.py:237-268 (geodesic angle in degrees, L2 translation)."""
    R_diff = pose_gt[:3, :3].T @ pose_noisy[:3, :3]
    trace = torch.trace(R_diff)
    angle_rad = torch.acos(torch.clamp((trace - 1) / 2, -1, 1))
    return {"rotation_error_deg": float(angle_rad * 180 / math.pi),
            "translation_error": float(torch.norm(pose_gt[:3, 3] - pose_noisy[:3, 3]))}


class _Bf16OperandLinear(nn.Module):
    """nn.Linear whose input and weight are rounded to bf16 (or fp16) (fp32 accumulate,
    fp32 bias): the operand precision of the MI355X 16-bit MFMA paths, used as their
    parity reference."""

    def __init__(self, lin: nn.Linear, dtype=torch.bfloat16):
        super().__init__()
        self.lin = lin
        self.dtype = dtype

    def forward(self, x):
        return F.linear(x.to(self.dtype).float(), self.lin.weight.to(self.dtype).float(), self.lin.bias)


def bf16_operand_nerf(model: "NeRF", dtype=torch.bfloat16) -> "NeRF":
    """Copy of an oracle NeRF whose MFMA layers (trunk, feature, dir) use bf16 (or fp16) operands."""
    import copy
    emu = copy.deepcopy(model)
    for i in range(len(emu.pts_linears)):
        emu.pts_linears[i] = _Bf16OperandLinear(emu.pts_linears[i], dtype)
    emu.feature_linear = _Bf16OperandLinear(emu.feature_linear, dtype)
    emu.dir_linear = _Bf16OperandLinear(emu.dir_linear, dtype)
    return emu


def fp16_operand_nerf(model: "NeRF") -> "NeRF":
    return bf16_operand_nerf(model, torch.float16)


# --------------------------------------------------------------------------
# Exact numerics model of the 16-bit MFMA path (parity reference at full size)
# --------------------------------------------------------------------------
class _GradRound(torch.autograd.Function):
    """Identity forward; the backward rounds the gradient to the 16-bit storage type
    (after scaling by ``scale``, a power of two, as the fp16 path does)."""

    @staticmethod
    def forward(ctx, z, dtype, scale):
        ctx.dtype, ctx.scale = dtype, scale
        return z.view_as(z)

    @staticmethod
    def backward(ctx, g):
        return (g * ctx.scale).to(ctx.dtype).float() / ctx.scale, None, None


class _FwdRound(torch.autograd.Function):
    """Round to the 16-bit operand type in the forward; the gradient passes through in
    fp32 untouched (a plain ``x.to(dt).float()`` would round the gradient too)."""

    @staticmethod
    def forward(ctx, x, dtype):
        return x.to(dtype).float()

    @staticmethod
    def backward(ctx, g):
        return g, None


class _HeadLinear(torch.autograd.Function):
    """A head layer (sigma, rgb): fp32 forward on the fp32 activations; backward
    dx = g W (fp32 g and W), dW = round16(g)^T round16(x), db = sum round16(g)."""

    @staticmethod
    def forward(ctx, x, weight, bias, dtype, scale):
        ctx.save_for_backward(x, weight)
        ctx.dtype, ctx.scale = dtype, scale
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        gr = (g * ctx.scale).to(ctx.dtype).float() / ctx.scale
        xr = x.to(ctx.dtype).float()
        return g @ weight, gr.t() @ xr, gr.sum(0), None, None


class MfmaEmulatedNeRF(nn.Module):
    """The NeRF forward/backward of the 16-bit MFMA kernels (csrc/mlp.hip), modelled
    value by value so that a comparison with them differs only in summation order:

    * every MFMA layer (trunk, feature, dir) takes 16-bit operands (activations and
      weights) with fp32 accumulation and an fp32 bias;
    * the sigma and rgb heads run in fp32 on the fp32 activations (VALU);
    * backward: each layer's dz (after its ReLU mask) is stored in 16 bit -- scaled by
      ``grad_scale`` (2^14 on the fp16 path) -- and both dX = W^T dz and dW = dz^T x use
      the stored value; the heads' dz feed dX in fp32 and dW in 16 bit, against the
      16-bit saved activations.

    Shares the base model's parameters (gradients land in them).  This models the
    build's arithmetic; the reference semantics it rounds are those of ``NeRF`` above."""

    def __init__(self, base: "NeRF", dtype=torch.bfloat16, grad_scale: float = 1.0):
        super().__init__()
        self.base = base
        self.dtype = dtype
        self.scale = float(grad_scale)

    def _lin(self, x, lin):
        dt = self.dtype
        return F.linear(_FwdRound.apply(x, dt), _FwdRound.apply(lin.weight, dt), lin.bias)

    def forward(self, x, d=None):
        b, dt, s = self.base, self.dtype, self.scale
        x_enc = b.pos_encoder(x)
        h = x_enc
        for i, layer in enumerate(b.pts_linears):
            h = F.relu(_GradRound.apply(self._lin(h, layer), dt, s))
            if i in b.config.skips:
                h = torch.cat([x_enc, h], dim=-1)
        sigma = F.relu(_HeadLinear.apply(h, b.sigma_linear.weight, b.sigma_linear.bias, dt, s))
        feats = _GradRound.apply(self._lin(h, b.feature_linear), dt, s)
        if b.config.use_view_dirs and d is not None:
            h_color = torch.cat([feats, b.dir_encoder(d)], dim=-1)
        else:
            h_color = feats
        h_color = F.relu(_GradRound.apply(self._lin(h_color, b.dir_linear), dt, s))
        rgb = torch.sigmoid(_HeadLinear.apply(h_color, b.rgb_linear.weight, b.rgb_linear.bias, dt, s))
        return rgb, sigma


def mfma_emulated_nerf(model: "NeRF", precision: str) -> nn.Module:
    """The exact numerics model for ModelConfig.precision 'bf16' or 'fp16' (fp16 backward
    on dz scaled by 2^14, include/nerf_hip.h NR_PREC_FP16)."""
    if precision == "bf16":
        return MfmaEmulatedNeRF(model, torch.bfloat16, 1.0)
    if precision == "fp16":
        return MfmaEmulatedNeRF(model, torch.float16, 2.0 ** 14)
    raise ValueError(precision)
