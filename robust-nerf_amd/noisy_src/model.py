"""
NeRF model — drop-in for ShawnnnLiu/Robust-NeRF ``noisy_src/model.py:20-221``.

``NeRF`` registers exactly the reference's submodules (``pts_linears.{i}``,
``sigma_linear``, ``feature_linear``, ``dir_linear``, ``rgb_linear``,
``pos_encoder.freq_bands``, ``dir_encoder.freq_bands``), built in the same order
with the same ``nn.Linear`` default init, so ``torch.manual_seed(s)`` gives the
reference's initial weights and checkpoints are interchangeable.

Underneath, the parameters are views into one flat fp32 buffer (the C-ABI
layout) and ``forward`` is a single fused HIP kernel (positional encoding, 8
trunk layers, skip concat, sigma/feature/dir/rgb heads) whose backward is the
fused dX chain + dW GEMM (csrc/mlp.hip).  ``ModelConfig.precision`` selects the
fp32 (parity) or bf16 MFMA path.
"""

from __future__ import annotations

import ctypes
import os
import weakref
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import _hip, ops
from ._hip import NrMlpConfig, call, ptr
from .config import ModelConfig


class PositionalEncoding(nn.Module):
    """Reference model.py:20-80: [x, sin(f0 x), cos(f0 x), ...], f = 2^k, no pi."""

    def __init__(self, num_freqs: int, include_input: bool = True, log_sampling: bool = True) -> None:
        super().__init__()
        self.num_freqs = num_freqs
        self.include_input = include_input
        self.log_sampling = log_sampling
        if log_sampling:
            freq_bands = 2.0 ** torch.linspace(0.0, num_freqs - 1, num_freqs)
        else:
            freq_bands = torch.linspace(1.0, 2.0 ** (num_freqs - 1), num_freqs)
        self.register_buffer("freq_bands", freq_bands)

    @property
    def output_dim(self) -> int:
        dim = 2 * self.num_freqs
        if self.include_input:
            dim += 1
        return dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.positional_encoding(x, self.num_freqs, self.include_input, self.log_sampling)


# NR_MLP_DENSE_BACKWARD=1 runs every 32-sample tile through the backward (the dense
# reference form, for A/B runs); by default tiles whose incoming gradient is exactly
# zero are skipped (csrc/mlp.hip, tile_flags_kernel: identical gradients)
_DENSE_BACKWARD = os.environ.get("NR_MLP_DENSE_BACKWARD", "0") not in ("", "0")


def _precision_code(p: str) -> int:
    if p == "fp32":
        return _hip.NR_PREC_FP32
    if p == "bf16":
        return _hip.NR_PREC_BF16
    if p == "fp16":
        return _hip.NR_PREC_FP16
    raise ValueError(f"ModelConfig.precision must be 'fp32', 'bf16' or 'fp16', got {p!r}")


class _MLPFunction(torch.autograd.Function):
    """Fused NeRF MLP forward/backward on MFMA (csrc/mlp.hip)."""

    @staticmethod
    def forward(ctx, x, d, net, *params):
        cfg = ctypes.byref(net._nr_cfg)
        flat = net._flat
        packed = net._packed_for_forward(params)
        xc = ops._c(x)
        dc = ops._c(d) if d is not None else None
        M = xc.shape[0]
        rgb = torch.empty(M, 3, device=xc.device, dtype=torch.float32)
        sigma = torch.empty(M, 1, device=xc.device, dtype=torch.float32)
        training = any(ctx.needs_input_grad)
        saved = None
        if training and M > 0:
            saved = torch.empty(int(_hip.load().nr_mlp_saved_bytes(cfg, M)), device=xc.device, dtype=torch.uint8)
        call("nr_mlp_forward", cfg, ptr(packed), ptr(flat), ptr(xc), ptr(dc), M, ptr(rgb), ptr(sigma), ptr(saved),
             _hip.stream_ptr(), tag=f"[M={M}]")
        if training:
            ctx.save_for_backward(xc, dc if dc is not None else xc.new_empty(0), rgb, sigma)
            ctx.has_d = dc is not None
            ctx.keep = (net, saved, packed, flat)
            ctx.shapes = [p.shape for p in params]
        return rgb, sigma

    @staticmethod
    def backward(ctx, g_rgb, g_sigma):
        xc, dc, rgb, sigma = ctx.saved_tensors
        net, saved, packed, flat = ctx.keep
        cfg = ctypes.byref(net._nr_cfg)
        M = xc.shape[0]
        dev = xc.device
        g_rgb = ops._c(g_rgb) if g_rgb is not None else torch.zeros(M, 3, device=dev)
        g_sigma = ops._c(g_sigma) if g_sigma is not None else torch.zeros(M, 1, device=dev)
        gflat = torch.empty(net._param_count, device=dev, dtype=torch.float32)
        g_x = torch.empty(M, 3, device=dev) if ctx.needs_input_grad[0] else None
        g_d = torch.empty(M, 3, device=dev) if (ctx.needs_input_grad[1] and ctx.has_d) else None
        if M > 0:
            ws = torch.empty(int(_hip.load().nr_mlp_workspace_bytes(cfg, M)), device=dev, dtype=torch.uint8)
            st, tag = _hip.stream_ptr(), f"[M={M}]"
            args = (cfg, ptr(packed), ptr(flat), ptr(xc), ptr(dc) if ctx.has_d else None, M, ptr(rgb), ptr(sigma),
                    ptr(saved), ptr(g_rgb), ptr(g_sigma), ptr(g_x), ptr(g_d), ptr(ws), st)
            # dX chain over the active tiles (dz images in HBM), then the dW GEMM over them
            call("nr_mlp_backward_dx", *args, tag=tag)
            call("nr_mlp_backward_dw", cfg, M, ptr(saved), ptr(ws), st, tag=tag)
            call("nr_mlp_backward_reduce", cfg, M, ptr(ws), ptr(gflat), st, tag=tag)
            if net._tile_counts is not None:
                # diagnostics (bench.py): the active-tile count this backward ran on
                off = int(_hip.load().nr_mlp_active_tiles_offset(cfg, M))
                net._tile_counts.append((M, ws[off:off + 4].view(torch.int32).clone()))
        else:
            gflat.zero_()
        net._last_gflat = gflat  # FusedAdam's fast path reads the flat gradient directly
        if net._grad_ready_hook is not None:
            # data parallel: start this net's gradient all-reduce now, overlapping the
            # rest of the backward (the fine net finishes before the coarse one)
            net._grad_ready_hook(gflat)
        grads = []
        off = 0
        for shape in ctx.shapes:
            n = shape.numel()
            grads.append(gflat[off:off + n].view(shape))
            off += n
        return (g_x, g_d, None, *grads)


def _check_supported(cfg: NrMlpConfig, config: ModelConfig, n_params: int) -> None:
    """Fail at construction, not at the first forward, for a ModelConfig the compiled
    kernels do not cover.  The fused MLP (csrc/mlp.hip) is specialised for the
    reference's width: hidden_dim 256 (8 MFMA row blocks of 32), pos_freqs <= 10
    (x_enc in 2 k-blocks), dir_freqs <= 4 (d_enc in 1 k-block); any depth 1..16 and
    any skip set.  The plan check is host code (nr_mlp_packed_bytes), so this runs
    without a GPU."""
    lib = _hip.load()
    if int(lib.nr_mlp_packed_bytes(ctypes.byref(cfg))) < 0:
        raise NotImplementedError(
            f"ModelConfig(hidden_dim={config.hidden_dim}, pos_freqs={config.pos_freqs}, "
            f"dir_freqs={config.dir_freqs}, num_hidden_layers={config.num_hidden_layers}, skips={config.skips}) "
            f"is outside the envelope of the compiled MI355X kernels: {_hip.last_error()} "
            "(supported: hidden_dim=256, pos_freqs<=10, dir_freqs<=4, 1..16 layers, any skips)")
    want = int(lib.nr_mlp_param_count(ctypes.byref(cfg)))
    if want != n_params:
        raise RuntimeError(f"NeRF parameter layout mismatch: module {n_params} vs kernel plan {want}")


# flat parameter buffer address -> the NeRF whose parameters it holds: FusedAdam
# (optim.py) finds the network whose packed images a step may refresh in place
_FLAT_OWNERS: "weakref.WeakValueDictionary[int, NeRF]" = weakref.WeakValueDictionary()


def flat_owner(pflat: torch.Tensor):
    """The NeRF whose flat parameter buffer starts at ``pflat`` (or None)."""
    return _FLAT_OWNERS.get(pflat.data_ptr())


class NeRF(nn.Module):
    """Reference model.py:83-196 (same submodules, parameter order and init)."""

    def __init__(self, config: ModelConfig | None = None) -> None:
        super().__init__()
        if config is None:
            config = ModelConfig()
        self.config = config
        self.pos_encoder = PositionalEncoding(num_freqs=config.pos_freqs, include_input=True)
        self.dir_encoder = PositionalEncoding(num_freqs=config.dir_freqs, include_input=True)
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

        skip_mask = 0
        for s in config.skips:
            skip_mask |= 1 << int(s)
        self._nr_cfg = NrMlpConfig(
            pos_freqs=config.pos_freqs, dir_freqs=config.dir_freqs, hidden=config.hidden_dim,
            n_layers=config.num_hidden_layers, skip_mask=skip_mask, use_view_dirs=int(bool(config.use_view_dirs)),
            precision=_precision_code(getattr(config, "precision", "fp32")),
            dense_backward=int(_DENSE_BACKWARD))
        self._param_count = sum(p.numel() for p in self.parameters())
        _check_supported(self._nr_cfg, config, self._param_count)
        self._flat: Optional[torch.Tensor] = None
        self._packed: Optional[torch.Tensor] = None
        self._packed_key = None
        self._table: Optional[torch.Tensor] = None
        self._last_gflat: Optional[torch.Tensor] = None  # the last backward's flat gradient
        # called with the flat gradient as soon as the backward has produced it
        self._grad_ready_hook = None
        # a list: every backward appends (M, its device count of active 32-sample tiles)
        self._tile_counts: Optional[list] = None
        self._tickets = {}  # device -> the persistent zeroed word of loss_ticket

    def loss_ticket(self, device) -> torch.Tensor:
        """A persistent device word, zero between launches, that the fused composite + MSE
        launch of this network's samples uses to sum its loss in the launch
        (ops.composite_mse).  One per network: the coarse and fine chains may run
        concurrently, each with its own."""
        t = self._tickets.get(device)
        if t is None:
            t = torch.zeros(4, device=device, dtype=torch.int32)
            self._tickets[device] = t
        return t

    # -- flat parameter buffer -------------------------------------------------
    @property
    def _param_list(self) -> List[nn.Parameter]:
        return list(self.parameters())

    def flat_params(self) -> torch.Tensor:
        """The flat fp32 buffer every parameter is a view of (C-ABI layout)."""
        self._ensure_flat()
        return self._flat

    def _ensure_flat(self, params: Optional[List[nn.Parameter]] = None) -> None:
        params = self._param_list if params is None else params
        flat = self._flat
        if flat is not None and flat.device == params[0].device:
            off = 0
            base = flat.data_ptr()
            ok = True
            for p in params:
                if p.data_ptr() != base + 4 * off or not p.is_contiguous():
                    ok = False
                    break
                off += p.numel()
            if ok:
                _FLAT_OWNERS[base] = self  # (again: e.g. after a deepcopy of the network)
                return
        dev = params[0].device
        _hip.require_device(params[0])
        flat = torch.empty(self._param_count, device=dev, dtype=torch.float32)
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + n].view(p.shape)
                off += n
        self._flat = flat
        self._packed_key = None
        _FLAT_OWNERS[flat.data_ptr()] = self

    def _packed_for_forward(self, params: Optional[List[nn.Parameter]] = None) -> torch.Tensor:
        params = self._param_list if params is None else params
        key = (self._flat.data_ptr(), tuple(p._version for p in params))
        if self._packed is None or self._packed_key != key or self._packed.device != self._flat.device:
            cfg = ctypes.byref(self._nr_cfg)
            nbytes = int(_hip.load().nr_mlp_packed_bytes(cfg))
            if nbytes < 0:
                raise RuntimeError(f"NeRF config unsupported by the HIP MLP: {_hip.last_error()}")
            # re-pack into the existing images when they fit: a captured hipGraph
            # (engine.GraphedTrainer) holds their address, so it stays valid
            if (self._packed is None or self._packed.numel() != nbytes
                    or self._packed.device != self._flat.device):
                self._packed = torch.empty(nbytes, device=self._flat.device, dtype=torch.uint8)
            call("nr_mlp_pack", cfg, ptr(self._flat), ptr(self._packed), _hip.stream_ptr())
            self._packed_key = key
        return self._packed

    def _pack_table(self) -> torch.Tensor:
        """The destination table of the packed images (nr_mlp_pack_table), built once per
        device: where every flat parameter lands in them, for the fused optimizer step."""
        t = self._table
        if t is None or t.device != self._flat.device:
            cfg = ctypes.byref(self._nr_cfg)
            nbytes = int(_hip.load().nr_mlp_pack_table_bytes(cfg))
            t = torch.empty(nbytes // 4, device=self._flat.device, dtype=torch.int32)
            call("nr_mlp_pack_table", cfg, ptr(t), _hip.stream_ptr())
            self._table = t
        return t

    def _fused_pack_target(self, pflat: torch.Tensor, params: Optional[List[nn.Parameter]] = None):
        """(table, packed) when an optimizer step over ``pflat`` -- exactly this network's
        flat parameters -- may refresh the packed images in its own launch (nr_adam_multi):
        the images must be current for the parameters before the step.  Else None (the
        next forward re-packs, as after any other change of the parameters)."""
        flat, packed = self._flat, self._packed
        if flat is None or packed is None or packed.device != flat.device:
            return None
        if pflat.data_ptr() != flat.data_ptr() or pflat.numel() != flat.numel():
            return None
        params = self._param_list if params is None else params
        if self._packed_key != (flat.data_ptr(), tuple(p._version for p in params)):
            return None
        return self._pack_table(), packed

    def _mark_packed_fresh(self, params: Optional[List[nn.Parameter]] = None) -> None:
        """After a fused step refreshed the images: they match the new parameter versions."""
        params = self._param_list if params is None else params
        self._packed_key = (self._flat.data_ptr(), tuple(p._version for p in params))

    def forward(self, x: torch.Tensor, d: torch.Tensor | None = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """x (N,3) positions, d (N,3) view dirs -> rgb (N,3) in [0,1], sigma (N,1) >= 0."""
        _hip.require_device(x, d)
        if self.config.use_view_dirs and d is None:
            # reference model.py:187-193 would feed 256 features to a 283-input layer
            raise ValueError("NeRF with use_view_dirs=True needs view directions d")
        params = self._param_list
        self._ensure_flat(params)
        return _MLPFunction.apply(x, d if self.config.use_view_dirs else None, self, *params)


def create_nerf(config: ModelConfig | None = None) -> Tuple[NeRF, NeRF | None]:
    """Reference model.py:199-221: coarse and fine networks of the same architecture."""
    if config is None:
        config = ModelConfig()
    model_coarse = NeRF(config)
    model_fine = NeRF(config)
    return model_coarse, model_fine
