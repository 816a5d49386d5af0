"""Host-side operators over the C ABI (include/nerf_hip.h), with autograd.

Each function allocates its outputs with the PyTorch caching allocator, hands
raw device pointers to one ``nr_*`` entry point on the current HIP stream and,
where the reference path is differentiable, is wrapped in a
``torch.autograd.Function`` whose backward is the matching HIP kernel.  There
is no CPU or eager-torch fallback: CPU tensors raise.
"""

from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import torch

from . import _hip
from ._hip import call, ptr

_f32 = torch.float32


def _stream() -> int:
    return _hip.stream_ptr()


def _c(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Contiguous fp32 view (no copy when already so)."""
    if t is None:
        return None
    if t.dtype != _f32:
        t = t.float()
    return t.contiguous()


def _check(*ts):
    _hip.require_device(*ts)


# ---------------------------------------------------------------- A1 / A2 ----
def ray_directions(H: int, W: int, focal: float, cx: float, cy: float, device) -> torch.Tensor:
    out = torch.empty(H, W, 3, device=device, dtype=_f32)
    if not out.is_cuda:
        _check(out)
    call("nr_ray_directions", H, W, float(focal), float(cx), float(cy), ptr(out), _stream())
    return out


class _GetRays(torch.autograd.Function):
    @staticmethod
    def forward(ctx, directions, c2w):
        d, c = _c(directions), _c(c2w)
        if c.shape[-2:] not in ((4, 4), (3, 4)):
            raise ValueError(f"get_rays: c2w must be (4,4) or (3,4), got {tuple(c.shape)}")
        shape = d.shape
        ro = torch.empty(shape, device=d.device, dtype=_f32)
        rd = torch.empty(shape, device=d.device, dtype=_f32)
        call("nr_get_rays", ptr(d), ptr(c), d.numel() // 3, ptr(ro), ptr(rd), _stream())
        ctx.save_for_backward(d, c)
        ctx.set_materialize_grads(False)
        return ro, rd

    @staticmethod
    def backward(ctx, g_ro, g_rd):
        d, c = ctx.saved_tensors
        if g_ro is None and g_rd is None:
            return None, None
        g4 = torch.zeros(4, 4, device=c.device, dtype=_f32)
        g_dirs = torch.empty_like(d) if (ctx.needs_input_grad[0] and g_rd is not None) else None
        ws = torch.empty(int(_hip.load().nr_get_rays_bwd_workspace_bytes()), device=c.device, dtype=torch.uint8)
        call("nr_get_rays_bwd", ptr(d), ptr(c), d.numel() // 3, ptr(_c(g_ro)), ptr(_c(g_rd)), ptr(g_dirs), ptr(g4),
             ptr(ws), _stream())
        g_c = g4[: c.shape[-2]] if ctx.needs_input_grad[1] else None
        if g_dirs is None and ctx.needs_input_grad[0]:
            g_dirs = torch.zeros_like(d)
        return g_dirs, g_c


def get_rays(directions: torch.Tensor, c2w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """rays.py:67-99; differentiable w.r.t. c2w and the directions, like the reference."""
    _check(directions, c2w)
    return _GetRays.apply(directions, c2w)


def _raise_if_flagged(flag: Optional[torch.Tensor], limit: int, what: str) -> None:
    """The validating mode's host side: one read of the device flag the kernel set."""
    if flag is not None and int(flag.item()):
        raise IndexError(f"{what} out of range for {limit} entries")


def gather_rays(idx, rays_o, rays_d, colors, validate: bool = False):
    """RaySampler batch assembly (data.py:264-321): the rows idx of the device ray table,
    all three arrays in one kernel.  ``validate`` (indices from a caller) raises
    IndexError, as the reference's tensor indexing does, for rows outside the table;
    the check rides in the gather kernel (one launch, one host read)."""
    _check(idx, rays_o, rays_d, colors)
    i = idx.to(torch.int64).contiguous()
    B = i.shape[0]
    out = [torch.empty(B, 3, device=i.device, dtype=_f32) for _ in range(3)]
    flag = torch.zeros(1, device=i.device, dtype=torch.int32) if validate else None
    call("nr_gather_rays", ptr(i), rays_o.shape[0], B, ptr(_c(rays_o)), ptr(_c(rays_d)), ptr(_c(colors)),
         ptr(out[0]), ptr(out[1]), ptr(out[2]), ptr(flag), _stream())
    _raise_if_flagged(flag, rays_o.shape[0], "ray index")
    return out


# ---------------------------------------------------------------- A5 / A9 / A10
def _pts_bwd(ctx, g_pts, z):
    """pts = o + d * z (rays.py:208 / :331): sum the sample gradients per ray."""
    g_o = g_d = None
    if g_pts is not None and (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]):
        B, S = z.shape
        g_o = torch.zeros(B, 3, device=z.device, dtype=_f32) if ctx.needs_input_grad[0] else None
        g_d = torch.zeros(B, 3, device=z.device, dtype=_f32) if ctx.needs_input_grad[1] else None
        call("nr_pts_bwd", ptr(_c(g_pts)), ptr(z), B, S, ptr(g_o), ptr(g_d), _stream())
    return g_o, g_d


def _viewdirs_bwd(ctx, g_vd, rd, S, g_d):
    """viewdirs = rays_d / |rays_d| per sample (rendering.py:165): accumulate into g_d."""
    if g_vd is None or not ctx.needs_input_grad[1]:
        return g_d
    if g_d is None:
        g_d = torch.zeros_like(rd)
    call("nr_viewdirs_bwd", ptr(rd), ptr(_c(g_vd)), rd.shape[0], S, ptr(g_d), _stream())
    return g_d


class _Stratified(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rays_o, rays_d, t_rand, near, far, lindisp, num_samples, with_vd):
        ro, rd = _c(rays_o), _c(rays_d)
        B = ro.shape[0]
        z = torch.empty(B, num_samples, device=ro.device, dtype=_f32)
        pts = torch.empty(B, num_samples, 3, device=ro.device, dtype=_f32)
        vd = torch.empty(B * num_samples, 3, device=ro.device, dtype=_f32) if with_vd else None
        tr = _c(t_rand)
        call("nr_stratified_sample", ptr(ro), ptr(rd), ptr(tr), float(near), float(far), int(bool(lindisp)), B,
             num_samples, ptr(z), ptr(pts), ptr(vd), _stream())
        ctx.save_for_backward(z, rd)
        ctx.mark_non_differentiable(z)
        ctx.set_materialize_grads(False)  # no zero-filled dL/dz launch per step
        return (pts, z, vd) if with_vd else (pts, z)

    @staticmethod
    def backward(ctx, g_pts, _g_z, g_vd=None):
        z, rd = ctx.saved_tensors
        g_o, g_d = _pts_bwd(ctx, g_pts, z)
        g_d = _viewdirs_bwd(ctx, g_vd, rd, z.shape[1], g_d)
        return g_o, g_d, None, None, None, None, None, None


def stratified_sample(rays_o, rays_d, near, far, num_samples, t_rand=None, lindisp=False, viewdirs=False):
    """Returns (pts (B,N,3), z (B,N)) -- and with ``viewdirs`` the normalised directions
    per sample (B*N,3) from the same launch; t_rand None -> no perturbation."""
    _check(rays_o, rays_d, t_rand)
    return _Stratified.apply(rays_o, rays_d, t_rand, near, far, lindisp, num_samples, bool(viewdirs))


def sample_pdf(bins, weights, num_samples, u=None):
    _check(bins, weights, u)
    b, w = _c(bins.detach()), _c(weights.detach())
    lead = b.shape[:-1]
    Nb = b.shape[-1]
    B = b.numel() // Nb
    uu = _c(u.detach()) if u is not None else None
    out = torch.empty(*lead, num_samples, device=b.device, dtype=_f32)
    call("nr_sample_pdf", ptr(b), ptr(w), ptr(uu), B, Nb, num_samples, ptr(out), _stream())
    return out


class _Hierarchical(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rays_o, rays_d, z_coarse, w_coarse, u, num_samples_fine, with_vd):
        ro, rd = _c(rays_o), _c(rays_d)
        zc, wc = _c(z_coarse), _c(w_coarse)
        B, Nc = zc.shape
        T = Nc + num_samples_fine
        zf = torch.empty(B, T, device=zc.device, dtype=_f32)
        pts = torch.empty(B, T, 3, device=zc.device, dtype=_f32)
        vd = torch.empty(B * T, 3, device=zc.device, dtype=_f32) if with_vd else None
        uu = _c(u)
        call("nr_sample_hierarchical", ptr(ro), ptr(rd), ptr(zc), ptr(wc), ptr(uu), B, Nc, num_samples_fine,
             ptr(zf), ptr(pts), ptr(vd), _stream())
        ctx.save_for_backward(zf, rd)
        ctx.mark_non_differentiable(zf)
        ctx.set_materialize_grads(False)
        return (pts, zf, vd) if with_vd else (pts, zf)

    @staticmethod
    def backward(ctx, g_pts, _g_z, g_vd=None):
        zf, rd = ctx.saved_tensors
        g_o, g_d = _pts_bwd(ctx, g_pts, zf)
        g_d = _viewdirs_bwd(ctx, g_vd, rd, zf.shape[1], g_d)
        return g_o, g_d, None, None, None, None, None


def sample_hierarchical(rays_o, rays_d, z_coarse, w_coarse, num_samples_fine, u=None, viewdirs=False):
    """Returns (pts_fine (B,Nc+Nf,3), z_fine (B,Nc+Nf)) -- and with ``viewdirs`` the
    normalised directions per sample from the same launch; u None -> det.  The fine
    depths are detached as in the reference (rays.py:325)."""
    _check(rays_o, rays_d, z_coarse, w_coarse, u)
    return _Hierarchical.apply(rays_o, rays_d, z_coarse.detach(), w_coarse.detach(),
                               u.detach() if u is not None else None, num_samples_fine, bool(viewdirs))


# ---------------------------------------------------------------- viewdirs ---
class _ExpandViewdirs(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rays_d, S):
        rd = _c(rays_d)
        B = rd.shape[0]
        out = torch.empty(B * S, 3, device=rd.device, dtype=_f32)
        call("nr_expand_viewdirs", ptr(rd), B, S, ptr(out), _stream())
        ctx.save_for_backward(rd)
        ctx.S = S
        return out

    @staticmethod
    def backward(ctx, g):
        (rd,) = ctx.saved_tensors
        g_rd = torch.zeros_like(rd)
        call("nr_viewdirs_bwd", ptr(rd), ptr(_c(g)), rd.shape[0], ctx.S, ptr(g_rd), _stream())
        return g_rd, None


def expand_viewdirs(rays_d: torch.Tensor, S: int) -> torch.Tensor:
    """normalize(rays_d) repeated for S samples per ray -> (B*S, 3) (rendering.py:165,182)."""
    _check(rays_d)
    return _ExpandViewdirs.apply(rays_d, S)


# ---------------------------------------------------------------- A6 ---------
class _PosEnc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, L, include_input, log_sampling):
        xc = _c(x)
        C = xc.shape[-1]
        M = xc.numel() // C
        D = (1 if include_input else 0) + 2 * L
        out = torch.empty(*xc.shape[:-1], C * D, device=xc.device, dtype=_f32)
        call("nr_positional_encoding", ptr(xc), M, C, L, int(include_input), int(log_sampling), ptr(out), _stream())
        ctx.save_for_backward(xc)
        ctx.args = (L, include_input, log_sampling)
        return out

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        L, inc, logs = ctx.args
        C = xc.shape[-1]
        gx = torch.empty_like(xc)
        call("nr_positional_encoding_bwd", ptr(xc), xc.numel() // C, C, L, int(inc), int(logs), ptr(_c(g)), ptr(gx),
             _stream())
        return gx, None, None, None


def positional_encoding(x, num_freqs, include_input=True, log_sampling=True):
    _check(x)
    return _PosEnc.apply(x, num_freqs, include_input, log_sampling)


# ---------------------------------------------------------------- A8 ---------
class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rgb, sigma, z, rays_d, noise, white):
        rgb, sigma, z, rd = _c(rgb), _c(sigma), _c(z), _c(rays_d)
        B, S = z.shape
        nz = _c(noise)
        rgb_map = torch.empty(B, 3, device=z.device, dtype=_f32)
        depth = torch.empty(B, device=z.device, dtype=_f32)
        acc = torch.empty(B, device=z.device, dtype=_f32)
        weights = torch.empty(B, S, device=z.device, dtype=_f32)
        call("nr_composite_fwd", ptr(rgb), ptr(sigma), ptr(z), ptr(rd), ptr(nz), B, S, int(white), ptr(rgb_map),
             ptr(depth), ptr(acc), ptr(weights), _stream())
        ctx.save_for_backward(rgb, sigma, z, rd, nz)
        ctx.white = white
        # unused outputs (depth/acc in training, the coarse weights) reach backward as
        # None, which the kernel reads as zero: no zero-filled tensors launched per step
        ctx.set_materialize_grads(False)
        return rgb_map, depth, acc, weights

    @staticmethod
    def backward(ctx, g_map, g_depth, g_acc, g_w):
        rgb, sigma, z, rd, nz = ctx.saved_tensors
        B, S = z.shape
        if g_map is None:
            g_map = torch.zeros(B, 3, device=z.device, dtype=_f32)
        g_rgb = torch.empty_like(rgb)
        g_sigma = torch.empty(B, S, device=z.device, dtype=_f32)
        g_rd = torch.zeros_like(rd) if ctx.needs_input_grad[3] else None
        call("nr_composite_bwd", ptr(rgb), ptr(sigma), ptr(z), ptr(rd), ptr(nz), B, S, int(ctx.white),
             ptr(_c(g_map)), ptr(_c(g_depth)), ptr(_c(g_acc)), ptr(_c(g_w)), ptr(g_rgb), ptr(g_sigma), ptr(g_rd),
             _stream())
        return g_rgb, g_sigma.view(sigma.shape), None, g_rd, None, None


def composite(rgb, sigma, z_vals, rays_d, noise=None, white_background=True):
    """raw2outputs core: rgb (B,S,3), sigma (B,S[,1]), z (B,S), rays_d (B,3)."""
    _check(rgb, sigma, z_vals, rays_d, noise)
    sig = sigma.reshape(z_vals.shape)
    return _Composite.apply(rgb, sig, z_vals, rays_d, noise, bool(white_background))


class _CompositeMSE(torch.autograd.Function):
    """raw2outputs + mean((rgb_map - target)^2) of one training step, one launch pair
    (nr_composite_mse): the forward also produces the gradient of ``grad_scale * loss``
    w.r.t. rgb / sigma (/ rays_d), which the backward hands over (bit-identical to the
    composite forward, MSE and composite backward run separately).  Gradients arriving
    at rgb_map / depth / acc / weights from elsewhere add a composite backward of their own."""

    @staticmethod
    def forward(ctx, rgb, sigma, z, rays_d, noise, target, white, grad_scale, ticket):
        rgb, sigma, z, rd, tgt = _c(rgb), _c(sigma), _c(z), _c(rays_d), _c(target)
        B, S = z.shape
        nz = _c(noise)
        dev = z.device
        rgb_map = torch.empty(B, 3, device=dev, dtype=_f32)
        depth = torch.empty(B, device=dev, dtype=_f32)
        acc = torch.empty(B, device=dev, dtype=_f32)
        weights = torch.empty(B, S, device=dev, dtype=_f32)
        loss = torch.empty((), device=dev, dtype=_f32)
        g_rgb = torch.empty_like(rgb)
        g_sigma = torch.empty(B, S, device=dev, dtype=_f32)
        g_rd = torch.zeros_like(rd) if ctx.needs_input_grad[3] else None
        ws = torch.empty(max(16, int(_hip.load().nr_composite_mse_workspace_bytes(B))), device=dev, dtype=torch.uint8)
        call("nr_composite_mse", ptr(rgb), ptr(sigma), ptr(z), ptr(rd), ptr(nz), ptr(tgt), B, S, int(white),
             float(grad_scale), ptr(rgb_map), ptr(depth), ptr(acc), ptr(weights), ptr(loss), ptr(g_rgb), ptr(g_sigma),
             ptr(g_rd), ptr(ticket), ptr(ws), _stream())
        ctx.save_for_backward(rgb, sigma, z, rd, nz, g_rgb, g_sigma, g_rd)
        ctx.white = white
        ctx.sigma_shape = sigma.shape
        ctx.set_materialize_grads(False)
        return loss, rgb_map, depth, acc, weights

    @staticmethod
    def backward(ctx, g_loss, g_map, g_depth, g_acc, g_w):
        rgb, sigma, z, rd, nz, g_rgb, g_sigma, g_rd = ctx.saved_tensors
        B, S = z.shape
        if g_loss is None:
            g_rgb, g_sigma = torch.zeros_like(g_rgb), torch.zeros_like(g_sigma)
            g_rd = torch.zeros_like(g_rd) if g_rd is not None else None
        elif g_loss.data_ptr() != _unit.get(g_loss.device, _NO_UNIT).data_ptr():
            g_rgb, g_sigma = g_rgb * g_loss, g_sigma * g_loss
            g_rd = g_rd * g_loss if g_rd is not None else None
        if any(t is not None for t in (g_map, g_depth, g_acc, g_w)):
            e_rgb, e_sigma = torch.empty_like(rgb), torch.empty(B, S, device=z.device, dtype=_f32)
            e_rd = torch.zeros_like(rd) if g_rd is not None else None
            gm = _c(g_map) if g_map is not None else torch.zeros(B, 3, device=z.device, dtype=_f32)
            call("nr_composite_bwd", ptr(rgb), ptr(sigma), ptr(z), ptr(rd), ptr(nz), B, S, int(ctx.white), ptr(gm),
                 ptr(_c(g_depth)), ptr(_c(g_acc)), ptr(_c(g_w)), ptr(e_rgb), ptr(e_sigma), ptr(e_rd), _stream())
            g_rgb, g_sigma = g_rgb + e_rgb, g_sigma + e_sigma
            g_rd = g_rd + e_rd if g_rd is not None else None
        return g_rgb, g_sigma.view(ctx.sigma_shape), None, g_rd, None, None, None, None, None


def composite_mse(rgb, sigma, z_vals, rays_d, target, noise=None, white_background=True, grad_scale=1.0,
                  ticket=None):
    """Training form of raw2outputs + the MSE loss against ``target`` (B,3): returns
    (loss, rgb_map, depth, acc, weights); the loss's gradient carries ``grad_scale``.
    ``ticket``: a persistent zeroed int32 device word (NeRF.loss_ticket) that lets the
    launch sum the loss itself; calls sharing it must not run concurrently."""
    _check(rgb, sigma, z_vals, rays_d, target, noise, ticket)
    sig = sigma.reshape(z_vals.shape)
    return _CompositeMSE.apply(rgb, sig, z_vals, rays_d, noise, target, bool(white_background), float(grad_scale),
                               ticket)


# ---------------------------------------------------------------- A3 / A4 ----
class _RaysFromPixels(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img_idx, pix, poses, H, W, focal, validate):
        img = img_idx.to(torch.int64).contiguous()
        px, ps = _c(pix), _c(poses)
        B = img.shape[0]
        ro = torch.empty(B, 3, device=px.device, dtype=_f32)
        rd = torch.empty(B, 3, device=px.device, dtype=_f32)
        flag = torch.zeros(1, device=px.device, dtype=torch.int32) if validate else None
        call("nr_rays_from_pixels_fwd", ptr(img), ptr(px), ptr(ps), ps.shape[0], H, W, float(focal), B, ptr(ro),
             ptr(rd), ptr(flag), _stream())
        _raise_if_flagged(flag, ps.shape[0], "image index")
        ctx.save_for_backward(img, px, ps)
        ctx.args = (H, W, float(focal))
        return ro, rd

    @staticmethod
    def backward(ctx, g_ro, g_rd):
        img, px, ps = ctx.saved_tensors
        H, W, focal = ctx.args
        B = img.shape[0]
        if g_ro is None:
            g_ro = torch.zeros(B, 3, device=px.device, dtype=_f32)
        g_poses = torch.zeros_like(ps)
        call("nr_rays_from_pixels_bwd", ptr(img), ptr(px), ptr(ps), ps.shape[0], H, W, focal, B, ptr(_c(g_ro)),
             ptr(_c(g_rd)), ptr(g_poses), _stream())
        return None, None, g_poses, None, None, None, None


def check_index_range(idx: torch.Tensor, limit: int, what: str = "index") -> None:
    """Raise IndexError (as torch indexing in the reference would) if any idx is outside
    [0, limit).  One device kernel plus one host read of the flag."""
    _check(idx)
    i = idx.to(torch.int64).contiguous()
    flag = torch.zeros(1, device=i.device, dtype=torch.int32)
    call("nr_check_index_range", ptr(i), i.numel(), int(limit), ptr(flag), _stream())
    if int(flag.item()):
        raise IndexError(f"{what} out of range for {limit} entries")


def rays_from_pixels(img_idx, pix, poses, H, W, focal, validate: bool = False):
    """get_rays_from_pixels (data_pose_opt.py:83-148) in one pass; poses indexed by img_idx.
    ``validate`` raises IndexError for an img_idx outside [0, poses.shape[0]) (the
    kernel's validating mode: same launch, one host read of its flag); unchecked
    out-of-range rays come out NaN and get no pose gradient."""
    _check(img_idx, pix, poses)
    return _RaysFromPixels.apply(img_idx, pix, poses, H, W, focal, bool(validate))


class _Se3Poses(torch.autograd.Function):
    @staticmethod
    def forward(ctx, init, rot, trans, indices, fixed_small_angle):
        ini = _c(init)
        r = _c(rot.detach()) if rot is not None else None
        t = _c(trans.detach()) if trans is not None else None
        idx = indices.to(torch.int64).contiguous() if indices is not None else None
        n = idx.shape[0] if idx is not None else ini.shape[0]
        out = torch.empty(n, 4, 4, device=ini.device, dtype=_f32)
        call("nr_se3_poses_fwd", ptr(ini), ptr(r), ptr(t), ptr(idx), n, ptr(out), _stream())
        ctx.save_for_backward(ini, r if r is not None else ini.new_empty(0), idx if idx is not None else ini.new_empty(0, dtype=torch.int64))
        ctx.flags = (r is not None, t is not None, idx is not None, n, bool(fixed_small_angle))
        return out

    @staticmethod
    def backward(ctx, g):
        ini, r, idx = ctx.saved_tensors
        has_r, has_t, has_idx, n, fixed = ctx.flags
        g_rot = torch.zeros(ini.shape[0], 3, device=ini.device, dtype=_f32) if (has_r and ctx.needs_input_grad[1]) else None
        g_trans = torch.zeros(ini.shape[0], 3, device=ini.device, dtype=_f32) if (has_t and ctx.needs_input_grad[2]) else None
        call("nr_se3_poses_bwd", ptr(ini), ptr(r) if has_r else None, ptr(idx) if has_idx else None, n,
             ini.shape[0], ptr(_c(g)), int(fixed), ptr(g_rot), ptr(g_trans), _stream())
        return None, g_rot, g_trans, None, None


def se3_poses(init_poses, rot_deltas=None, trans_deltas=None, indices=None, fixed_small_angle=False):
    _check(init_poses, rot_deltas, trans_deltas, indices)
    return _Se3Poses.apply(init_poses, rot_deltas, trans_deltas, indices, fixed_small_angle)


# ---------------------------------------------------------------- loss -------
def mse_loss_and_grad(pred, target, scale=1.0):
    """(loss (device scalar), d loss/d pred * scale) for mean((pred-target)^2)."""
    _check(pred, target)
    p, t = _c(pred), _c(target)
    loss = torch.empty((), device=p.device, dtype=_f32)
    g = torch.empty_like(p)
    call("nr_mse_fwd_bwd", ptr(p), ptr(t), p.shape[0], float(scale), ptr(loss), ptr(g), _stream())
    return loss, g


# ---------------------------------------------------------------- optimizer --
_sumsq_ws = {}


def sumsq_into(x: torch.Tensor, acc: torch.Tensor) -> None:
    """acc += sum(x^2) (fixed-order two-pass reduction: bit-reproducible)."""
    ws = _sumsq_ws.get(x.device)
    if ws is None:
        ws = torch.empty(int(_hip.load().nr_sumsq_workspace_bytes()), device=x.device, dtype=torch.uint8)
        _sumsq_ws[x.device] = ws  # stream-ordered reuse: every call runs on the current stream
    call("nr_sumsq", ptr(x), x.numel(), ptr(acc), ptr(ws), _stream())


def adam_step(p, g, m, v, lr, beta1, beta2, eps, step, sumsq=None, max_norm=1.0):
    call("nr_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr), float(beta1), float(beta2), float(eps),
         int(step), ptr(sumsq), float(max_norm), _stream())


MAX_ADAM_SPANS = 8


def sumsq_partials(xs, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The fixed-order partial sums of squares over the concatenation of the fp32 device
    buffers ``xs`` (one clip group, <= 8 buffers): a (256,) device tensor that
    ``adam_multi`` turns into the clip coefficient (no zeroed accumulator, one launch)."""
    if not 1 <= len(xs) <= MAX_ADAM_SPANS:
        raise ValueError(f"sumsq_partials: 1..{MAX_ADAM_SPANS} buffers, got {len(xs)}")
    _check(*xs)
    if out is None:
        out = torch.empty(int(_hip.load().nr_sumsq_workspace_bytes()) // 4, device=xs[0].device, dtype=_f32)
    ptrs = (ctypes.c_void_p * len(xs))(*[ptr(x) for x in xs])
    ns = (ctypes.c_int64 * len(xs))(*[x.numel() for x in xs])
    call("nr_sumsq_partials", ptrs, ns, len(xs), ptr(out), _stream())
    return out


def adam_sched_values(lr: float, beta1: float, beta2: float, step: int) -> Tuple[float, float]:
    """(lr / (1 - beta1^step), sqrt(1 - beta2^step)): the two step-dependent Adam scalars,
    in double as nr_adam_step / torch's Adam compute them (to be rounded to fp32)."""
    import math
    return lr / (1.0 - beta1 ** step), math.sqrt(1.0 - beta2 ** step)


def adam_multi(spans, lr, beta1, beta2, eps, step, sched: Optional[torch.Tensor] = None) -> None:
    """torch.optim.Adam over up to 8 flat buffers in one launch.  Each span is a dict with
    p, g, m, v (fp32 device buffers of one size), optional ``partials`` (the span's clip
    group, from ``sumsq_partials``) and ``max_norm``, and optional ``table`` / ``packed``
    (an MLP's destination table and images, refreshed in the same launch).  ``sched``:
    a device fp32 pair (``adam_sched_values``) the kernel reads instead of lr / step."""
    if not 1 <= len(spans) <= MAX_ADAM_SPANS:
        raise ValueError(f"adam_multi: 1..{MAX_ADAM_SPANS} spans, got {len(spans)}")
    arr = (_hip.NrAdamSpan * len(spans))()
    for k, sp in enumerate(spans):
        n = sp["p"].numel()
        if any(sp[x].numel() != n for x in ("g", "m", "v")):
            raise ValueError("adam_multi: p, g, m, v must have the same size")
        arr[k] = _hip.NrAdamSpan(ptr(sp["p"]), ptr(sp["g"]), ptr(sp["m"]), ptr(sp["v"]), n,
                                 ptr(sp.get("partials")), float(sp.get("max_norm", 1.0)),
                                 ptr(sp.get("table")), ptr(sp.get("packed")))
    call("nr_adam_multi", arr, len(spans), float(lr), float(beta1), float(beta2), float(eps), int(step), ptr(sched),
         _stream())


class _MSE(torch.autograd.Function):
    """mean((pred - target)^2) (train.py:89); the gradient is produced in the same kernel,
    times ``grad_scale`` (data parallelism folds its 1/world into it: the all-reduced
    SUM of the ranks' gradients is then the global-batch mean with no extra launch)."""

    @staticmethod
    def forward(ctx, pred, target, grad_scale):
        loss, g = mse_loss_and_grad(pred, target, grad_scale)
        ctx.save_for_backward(g)
        return loss

    @staticmethod
    def backward(ctx, gl):
        (g,) = ctx.saved_tensors
        # seeded by unit_grad(): gl is exactly 1.0, so g * gl == g (no multiply launch)
        if gl.data_ptr() == _unit.get(gl.device, _NO_UNIT).data_ptr():
            return g, None, None
        return g * gl, None, None


_unit = {}
_NO_UNIT = torch.empty(0)


def unit_grad(device) -> torch.Tensor:
    """A cached device scalar 1.0 to seed ``loss.backward(unit_grad(dev))``: no fill
    kernel for the seed, and the MSE backward (reached through sums of losses, whose
    backward forwards the seed tensor itself) skips its multiply by it.  Never write
    into it."""
    u = _unit.get(device)
    if u is None:
        u = torch.ones((), device=device, dtype=_f32)
        _unit[device] = u
    return u


def mse_loss(pred: torch.Tensor, target: torch.Tensor, grad_scale: float = 1.0) -> torch.Tensor:
    """The loss value is always the plain mean; only its gradient carries ``grad_scale``."""
    _check(pred, target)
    return _MSE.apply(pred, target, float(grad_scale))
