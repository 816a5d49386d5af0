"""The C-ABI library loads inside a torch process and its kernels run on torch's
stream (torch bundles HIP 7.0; the library is built by ROCm 7.2 hipcc)."""
import numpy as np
import pytest
import torch

from noisy_src import _hip

_hip.load(require_all=False)  # the full ABI is checked in test_abi.py


@pytest.mark.gpu
def test_probe_fill_on_torch_stream():
    out = torch.empty(1000, device="cuda")
    _hip.call("nr_probe_fill", _hip.ptr(out), 1000, 3.0, _hip.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), torch.arange(1000, dtype=torch.float32) + 3.0)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [0, 1])
def test_mfma_lane_maps(kind):
    g = torch.Generator().manual_seed(kind)
    K = 16 if kind == 0 else 2
    # small integers: exact in bf16, asymmetric A and B (guide §3: A=I checks miss transposes)
    A = torch.randint(-4, 5, (32, K), generator=g).float()
    B = torch.randint(-4, 5, (K, 32), generator=g).float()
    D = torch.empty(32, 32, device="cuda")
    Ad, Bd = A.cuda(), B.cuda()  # keep device copies alive until the kernel has run
    _hip.call("nr_probe_mfma", kind, _hip.ptr(Ad), _hip.ptr(Bd), _hip.ptr(D), _hip.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(D.cpu(), A @ B)
