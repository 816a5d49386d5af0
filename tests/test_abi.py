"""CPU: the C-ABI library loads and exports every entry point include/nerf_hip.h declares,
and the ctypes signature table covers exactly those symbols (no compute calls)."""
import re
import subprocess
from pathlib import Path

import pytest

from noisy_src import _hip

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "nerf_hip.h"


def _declared():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nr_[a-z0-9_]+)\s*\(", text)))


def test_header_and_ctypes_table_agree():
    assert _declared() == sorted(_hip.exported_symbols())


def test_library_exports_every_symbol():
    lib = _hip.lib_path()
    if not lib.exists():
        pytest.skip("library not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(nr_[a-z0-9_]+)", out))
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing
    _hip._lib = None
    _hip.load(require_all=True)  # dlopen + resolve all, no kernel launch


def test_no_cpu_fallback():
    import torch
    with pytest.raises(RuntimeError, match="no CPU fallback|CPU"):
        _hip.ptr(torch.zeros(3))


def test_plan_sizes_match_reference_model():
    """nr_mlp_param_count on the default config is the reference's 595,844 (summary.json)."""
    import ctypes
    lib = _hip.lib_path()
    if not lib.exists():
        pytest.skip("library not built")
    L = _hip.load()
    cfg = _hip.NrMlpConfig(pos_freqs=10, dir_freqs=4, hidden=256, n_layers=8, skip_mask=1 << 4, use_view_dirs=1,
                           precision=_hip.NR_PREC_BF16)
    assert L.nr_mlp_param_count(ctypes.byref(cfg)) == 595844
    assert L.nr_mlp_packed_bytes(ctypes.byref(cfg)) > 0
    assert L.nr_mlp_saved_bytes(ctypes.byref(cfg), 1000) > 0
    bad = _hip.NrMlpConfig(pos_freqs=10, dir_freqs=4, hidden=128, n_layers=8, skip_mask=16, use_view_dirs=1,
                           precision=0)
    assert L.nr_mlp_param_count(ctypes.byref(bad)) == -1
    assert "hidden_dim" in _hip.last_error()


def test_struct_layouts_match_header():
    """The ctypes mirrors list the header's struct fields in order (NrMlpConfig gained
    dense_backward in ABI 5)."""
    text = HEADER.read_text()
    for name, mirror in (("NrMlpConfig", _hip.NrMlpConfig), ("NrAdamSpan", _hip.NrAdamSpan)):
        body = re.search(r"typedef struct " + name + r" \{(.*?)\} " + name + ";", text, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        assert re.findall(r"(\w+)\s*;", body) == [f[0] for f in mirror._fields_], name


def test_abi_version():
    lib = _hip.lib_path()
    if not lib.exists():
        pytest.skip("library not built")
    assert _hip.load().nr_abi_version() == 5
