"""tools/prof_summary.py attributes every fused-MLP launch to its sample count M: the
forward / dX grids give it, dW / the reduction / the input gradients follow the
backward launch of the same net; and a re-summary under an overridden source hash is
marked as such (bench.py refuses it)."""

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import prof_summary  # noqa: E402

FWD_T = "nr::mlp_fwd_rbm_kernel<1, 2, 1, true>(nr::RbmArgs)"
FWD_I = "nr::mlp_fwd_rbm_kernel<1, 2, 1, false>(nr::RbmArgs)"
DX = "nr::mlp_bwd_rbm_kernel<1>(nr::BwdrArgs)"
DW = "nr::mlp_dw_kernel<1>(nr::DwArgs)"
RED = "nr::mlp_dw_reduce_kernel(nr::ReduceArgs)"
FLAGS = "nr::tile_flags_kernel(float const*, float const*, long, long, int, unsigned char*)"


def grid_of(M):
    return M // 32 * 64  # one 32-sample tile per wave


def test_split_backward_and_inference_forwards():
    t = prof_summary.MTracker()
    coarse, fine = 262_144, 786_432
    seq = [(FWD_I, grid_of(4096)),  # an eval forward: no backward follows
           (FWD_T, grid_of(coarse)), (FWD_T, grid_of(fine)), (FLAGS, 98_304), (DX, grid_of(fine)), (DW, 128_000),
           (RED, 1), (FLAGS, 32_768), (DX, grid_of(coarse)), (DW, 128_000), (RED, 1)]
    got = [t(n, g) for n, g in seq]
    assert got == [4096, coarse, fine, 0, fine, fine, fine, 0, coarse, coarse, coarse]


def test_source_hash_override_is_recorded(monkeypatch):
    monkeypatch.delenv("NR_SOURCE_HASH", raising=False)
    real = prof_summary.source_hash()
    assert real == prof_summary.computed_hash()
    monkeypatch.setenv("NR_SOURCE_HASH", "0123456789ab")
    assert prof_summary.source_hash() == "0123456789ab" != prof_summary.computed_hash()
