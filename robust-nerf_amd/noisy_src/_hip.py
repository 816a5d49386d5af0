"""ctypes binding of the gfx950 C-ABI library ``lib/libnerf_hip.so``.

The library is declared in ``include/nerf_hip.h``.  ``torch`` is imported
before the library is loaded: torch ships its own ``libamdhip64.so.7`` and the
library's DT_NEEDED entry of the same SONAME then binds to that already-loaded
runtime, so torch's streams and allocations are valid inside our kernels.

There is no fallback: if the library is missing, or a tensor handed to it is
not a contiguous tensor on a ROCm device, the call raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import torch

# NR_HIP_LIB selects another build of the same library (kernel-variant experiments).
_LIB_PATH = Path(os.environ.get("NR_HIP_LIB") or Path(__file__).resolve().parent / "lib" / "libnerf_hip.so")

c_vp = ctypes.c_void_p
c_i = ctypes.c_int
c_i64 = ctypes.c_int64
c_f = ctypes.c_float
c_d = ctypes.c_double
c_u32 = ctypes.c_uint32


class NrMlpConfig(ctypes.Structure):
    """Mirror of ``struct NrMlpConfig`` (include/nerf_hip.h)."""

    _fields_ = [
        ("pos_freqs", c_i),
        ("dir_freqs", c_i),
        ("hidden", c_i),
        ("n_layers", c_i),
        ("skip_mask", c_u32),
        ("use_view_dirs", c_i),
        ("precision", c_i),
        ("dense_backward", c_i),
    ]


class NrAdamSpan(ctypes.Structure):
    """Mirror of ``struct NrAdamSpan`` (include/nerf_hip.h)."""

    _fields_ = [
        ("params", c_vp),
        ("grads", c_vp),
        ("exp_avg", c_vp),
        ("exp_avg_sq", c_vp),
        ("n", c_i64),
        ("sumsq_partials", c_vp),
        ("max_norm", c_f),
        ("pack_table", c_vp),
        ("packed", c_vp),
    ]


NR_PREC_FP32 = 0
NR_PREC_BF16 = 1
NR_PREC_FP16 = 2
_cfg_p = ctypes.POINTER(NrMlpConfig)

# name -> (restype, argtypes); mirrors include/nerf_hip.h one to one.
_SIGNATURES = {
    "nr_last_error": (ctypes.c_char_p, []),
    "nr_abi_version": (c_i, []),
    "nr_probe_fill": (c_i, [c_vp, c_i, c_f, c_vp]),
    "nr_probe_mfma": (c_i, [c_i, c_vp, c_vp, c_vp, c_vp]),
    "nr_ray_directions": (c_i, [c_i, c_i, c_f, c_f, c_f, c_vp, c_vp]),
    "nr_get_rays": (c_i, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "nr_get_rays_bwd_workspace_bytes": (c_i64, []),
    "nr_get_rays_bwd": (c_i, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nr_rays_from_pixels_fwd": (c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_i, c_f, c_i, c_vp, c_vp, c_vp, c_vp]),
    "nr_rays_from_pixels_bwd": (c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_i, c_f, c_i, c_vp, c_vp, c_vp, c_vp]),
    "nr_se3_poses_fwd": (c_i, [c_vp, c_vp, c_vp, c_vp, c_i, c_vp, c_vp]),
    "nr_check_index_range": (c_i, [c_vp, c_i, c_i, c_vp, c_vp]),
    "nr_se3_poses_bwd": (c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_vp, c_i, c_vp, c_vp, c_vp]),
    "nr_gather_rays": (c_i, [c_vp, c_i64, c_i, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nr_stratified_sample": (c_i, [c_vp, c_vp, c_vp, c_f, c_f, c_i, c_i, c_i, c_vp, c_vp, c_vp, c_vp]),
    "nr_positional_encoding": (c_i, [c_vp, c_i64, c_i, c_i, c_i, c_i, c_vp, c_vp]),
    "nr_positional_encoding_bwd": (c_i, [c_vp, c_i64, c_i, c_i, c_i, c_i, c_vp, c_vp, c_vp]),
    "nr_sample_pdf": (c_i, [c_vp, c_vp, c_vp, c_i, c_i, c_i, c_vp, c_vp]),
    "nr_sample_hierarchical": (c_i, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_vp, c_vp, c_vp, c_vp]),
    "nr_composite_fwd": (c_i, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nr_composite_bwd": (c_i, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_vp, c_vp, c_vp, c_vp,
                               c_vp, c_vp, c_vp, c_vp]),
    "nr_mlp_param_count": (c_i64, [_cfg_p]),
    "nr_mlp_packed_bytes": (c_i64, [_cfg_p]),
    "nr_mlp_saved_bytes": (c_i64, [_cfg_p, c_i64]),
    "nr_mlp_workspace_bytes": (c_i64, [_cfg_p, c_i64]),
    "nr_mlp_pack": (c_i, [_cfg_p, c_vp, c_vp, c_vp]),
    "nr_mlp_forward": (c_i, [_cfg_p, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "nr_mlp_backward": (c_i, [_cfg_p, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp,
                              c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nr_mlp_backward_dx": (c_i, [_cfg_p, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp, c_vp]),
    "nr_mlp_backward_dw": (c_i, [_cfg_p, c_i64, c_vp, c_vp, c_vp]),
    "nr_mlp_backward_reduce": (c_i, [_cfg_p, c_i64, c_vp, c_vp, c_vp]),
    "nr_mlp_active_tiles_offset": (c_i64, [_cfg_p, c_i64]),
    "nr_sumsq_workspace_bytes": (c_i64, []),
    "nr_sumsq": (c_i, [c_vp, c_i64, c_vp, c_vp, c_vp]),
    "nr_adam_step": (c_i, [c_vp, c_vp, c_vp, c_vp, c_i64, c_d, c_d, c_d, c_d, c_i64, c_vp, c_f, c_vp]),
    "nr_sumsq_partials": (c_i, [c_vp, c_vp, c_i, c_vp, c_vp]),
    "nr_adam_multi": (c_i, [ctypes.POINTER(NrAdamSpan), c_i, c_d, c_d, c_d, c_d, c_i64, c_vp, c_vp]),
    "nr_mlp_pack_table_bytes": (c_i64, [_cfg_p]),
    "nr_mlp_pack_table": (c_i, [_cfg_p, c_vp, c_vp]),
    "nr_expand_viewdirs": (c_i, [c_vp, c_i, c_i, c_vp, c_vp]),
    "nr_pts_bwd": (c_i, [c_vp, c_vp, c_i, c_i, c_vp, c_vp, c_vp]),
    "nr_viewdirs_bwd": (c_i, [c_vp, c_vp, c_i, c_i, c_vp, c_vp]),
    "nr_composite_mse_workspace_bytes": (c_i64, [c_i]),
    "nr_composite_mse": (c_i, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i, c_i, c_i, c_f, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "nr_mse_fwd_bwd": (c_i, [c_vp, c_vp, c_i, c_f, c_vp, c_vp, c_vp]),
}

_lib: Optional[ctypes.CDLL] = None


def lib_path() -> Path:
    return _LIB_PATH


def load(require_all: bool = True) -> ctypes.CDLL:
    """Load (once) and return the library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not _LIB_PATH.exists():
        raise RuntimeError(
            f"noisy_src: HIP library {_LIB_PATH} not built; run `make -C robust-nerf_amd` "
            "(or __graft_entry__.build()). There is no CPU fallback."
        )
    lib = ctypes.CDLL(str(_LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if require_all:
                raise RuntimeError(f"noisy_src: {_LIB_PATH} does not export {name}")
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def exported_symbols() -> list:
    return list(_SIGNATURES)


def last_error() -> str:
    msg = load().nr_last_error()
    return msg.decode() if msg else ""


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device: Optional[torch.device] = None) -> int:
    """The current HIP stream of ``device`` (default: the current device) as an int --
    the raw accessor, without building a torch.cuda.Stream object per launch."""
    if _raw_stream is not None and device is None:
        return _raw_stream(torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


class CallTimer:
    """Brackets selected entry points with HIP events on the launching stream (the
    current torch stream the kernels run on), for per-launch durations in bench.py."""

    def __init__(self, names, keys=None):
        self.names = set(names)
        self.keys = None if keys is None else set(keys)  # optional: only these name+tag keys
        self.events = {}

    def wants(self, key) -> bool:
        return self.keys is None or key in self.keys

    def record(self, key, fn):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn()
        e.record()
        self.events.setdefault(key, []).append((s, e))
        return rc

    def summary(self):
        """key -> (launches, mean ms); call after torch.cuda.synchronize()."""
        return {k: (len(v), sum(a.elapsed_time(b) for a, b in v) / len(v)) for k, v in self.events.items()}


_timer: Optional[CallTimer] = None


def set_timer(timer: Optional[CallTimer]) -> None:
    global _timer
    _timer = timer


def call(name: str, *args, tag: str = "") -> int:
    """Invoke an ``nr_*`` entry point and raise RuntimeError on a non-zero code."""
    fn = getattr(load(), name)
    if _timer is not None and name in _timer.names and _timer.wants(f"{name}{tag}"):
        rc = _timer.record(f"{name}{tag}", lambda: fn(*args))
    else:
        rc = fn(*args)
    if isinstance(rc, int) and fn.restype is c_i and rc != 0:
        raise RuntimeError(f"{name} failed (code {rc}): {last_error()}")
    return rc


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    """Device pointer of a contiguous ROCm tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError(
            "noisy_src HIP path: tensor is on the CPU; this framework has no CPU fallback "
            "(move the inputs to a ROCm device)"
        )
    if not t.is_contiguous():
        raise RuntimeError("noisy_src HIP path: tensor must be contiguous")
    return t.data_ptr()


def require_device(*tensors: Optional[torch.Tensor]) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                "noisy_src HIP path: got a CPU tensor; there is no CPU fallback "
                "(this is the MI355X framework — run on a ROCm device)"
            )
