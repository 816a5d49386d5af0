"""Data-parallel gradient path on CPU (gloo, world size 2): the bucketed async
all-reduce that the Trainer hooks into each network's backward."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from noisy_src.engine import GradAllReducer


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        fine = torch.randn(595_844, generator=g)
        coarse = torch.randn(595_844, generator=g)
        red = GradAllReducer(dist.group.WORLD)
        red.launch(fine)    # fine net's backward finishes first
        red.launch(coarse)  # then the coarse net's
        red.finish()
        out[rank] = (fine.clone(), coarse.clone())
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_is_the_mean_on_every_rank():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    exp_f = sum(torch.randn(595_844, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)) / world
    gens = [torch.Generator().manual_seed(100 + r) for r in range(world)]
    for gg in gens:
        torch.randn(595_844, generator=gg)
    exp_c = sum(torch.randn(595_844, generator=gg) for gg in gens) / world
    for r in range(world):
        f, c = res[r]
        assert torch.allclose(f, exp_f, rtol=0, atol=1e-6)
        assert torch.allclose(c, exp_c, rtol=0, atol=1e-6)
    # every rank holds bit-identical averaged gradients (identical Adam updates follow)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
