"""tools/prof_summary.py attributes every fused-MLP launch to its sample count M
(the layer-pipelined backward's grid is pipelines x stages, so its
M must come from the training forward of the same net, not from the last launch)."""

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import prof_summary  # noqa: E402

FWD_T = "nr::mlp_fwd_rbm_kernel<1, 2, 1, true>(nr::RbmArgs)"
FWD_I = "nr::mlp_fwd_rbm_kernel<1, 2, 1, false>(nr::RbmArgs)"
PIPE = "nr::mlp_bwd_pipe_kernel<1, 2, 1, 2>(nr::PipeArgs)"
DX = "nr::mlp_bwd_rbm_kernel<1>(nr::BwdrArgs)"
DW = "nr::mlp_dw_kernel<1>(nr::DwArgs)"
RED = "nr::mlp_dw_reduce_kernel(nr::ReduceArgs)"


def grid_of(M):
    return M // 32 * 64  # one 32-sample tile per wave


def test_fused_backward_takes_its_own_nets_M():
    t = prof_summary.MTracker()
    coarse, fine = 262_144, 786_432
    seq = [(FWD_T, grid_of(coarse)), (FWD_T, grid_of(fine)), (PIPE, 64_000), (RED, 595_968),
           (PIPE, 64_000), (RED, 595_968)]
    got = [t(n, g) for n, g in seq]
    assert got == [coarse, fine, fine, fine, coarse, coarse]


def test_split_backward_and_inference_forwards():
    t = prof_summary.MTracker()
    coarse, fine = 262_144, 786_432
    seq = [(FWD_I, grid_of(4096)),  # an eval forward: no backward follows
           (FWD_T, grid_of(coarse)), (FWD_T, grid_of(fine)), (DX, grid_of(fine)), (DW, 128_000), (RED, 1),
           (DX, grid_of(coarse)), (DW, 128_000), (RED, 1),
           # next step, fused
           (FWD_T, grid_of(coarse)), (FWD_T, grid_of(fine)), (PIPE, 64_000), (PIPE, 64_000)]
    got = [t(n, g) for n, g in seq]
    assert got == [4096, coarse, fine, fine, fine, fine, coarse, coarse, coarse, coarse, fine, fine, coarse]
