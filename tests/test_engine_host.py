"""Host logic of engine.py that needs no GPU."""

import torch
import torch.nn as nn


class _Net(nn.Module):
    """Stand-in with the attributes _adopt_reduced_grad reads: equal-sized parameter sets,
    .grad tensors that are NOT views of the flat gradient (the copy fallback), and the
    last backward's flat gradient."""

    def __init__(self, flat):
        super().__init__()
        self.a = nn.Parameter(torch.zeros(3, 2))
        self.b = nn.Parameter(torch.zeros(4))
        self._param_count = 10
        self._last_gflat = flat
        for p in self.parameters():
            p.grad = torch.full_like(p, -1.0)


def test_reduced_grad_fallback_picks_each_nets_own_flat():
    """Coarse and fine nets have equal parameter counts; with the coarse chain on a second
    stream the coarse all-reduce can be launched first, so the pending list's order says
    nothing about ownership (the copy fallback used to match by size only, and removed
    the match with list.remove, whose == on tensors is elementwise)."""
    from noisy_src.engine import _adopt_reduced_grad
    f_coarse = torch.arange(10, dtype=torch.float32)
    f_fine = torch.arange(10, dtype=torch.float32) + 100
    coarse, fine = _Net(f_coarse), _Net(f_fine)
    flats = [f_fine, f_coarse]  # fine first, as in the one-stream step
    _adopt_reduced_grad(coarse, flats)
    _adopt_reduced_grad(fine, flats)
    assert torch.equal(torch.cat([coarse.a.grad.reshape(-1), coarse.b.grad]), f_coarse)
    assert torch.equal(torch.cat([fine.a.grad.reshape(-1), fine.b.grad]), f_fine)
    assert flats == []
