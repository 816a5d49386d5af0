"""GPU: the fused optimizer tail (nr_sumsq_partials + nr_adam_multi with the pack table).

The step must (1) update parameters exactly as torch.optim.Adam after
clip_grad_norm_ (train.py:112-117; train_pose_opt.py:398-404 per-network clips), and
(2) leave every network's packed MFMA images byte-identical to a fresh nr_mlp_pack of
the updated parameters, for every precision and for non-default model configs, so the
forward after it may skip the re-pack."""
import ctypes

import pytest
import torch


pytestmark = pytest.mark.gpu
DEV = "cuda"

CONFIGS = {
    "bf16": dict(precision="bf16"),
    "fp16": dict(precision="fp16"),
    "fp32": dict(precision="fp32"),
    "bf16_no_view_dirs": dict(precision="bf16", use_view_dirs=False),
    "fp16_depth7_skips2_5": dict(precision="fp16", num_hidden_layers=7, skips=(2, 5)),
    "bf16_depth1": dict(precision="bf16", num_hidden_layers=1, skips=()),
}


def _fresh_pack(net):
    """nr_mlp_pack of the current parameters over a copy of the images (so the alignment
    gaps nr_mlp_pack never writes compare equal)."""
    from noisy_src import _hip
    from noisy_src._hip import call, ptr
    cfg = ctypes.byref(net._nr_cfg)
    out = net._packed.clone()
    call("nr_mlp_pack", cfg, ptr(net._flat), ptr(out), _hip.stream_ptr())
    return out


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_fused_step_matches_torch_adam_and_repack(name):
    from noisy_src.config import ModelConfig
    from noisy_src.model import NeRF
    from noisy_src.optim import FusedAdam
    cfg = ModelConfig(**CONFIGS[name])
    torch.manual_seed(3)
    nets = [NeRF(cfg).to(DEV), NeRF(cfg).to(DEV)]  # coarse + fine: two spans, one clip group
    ref_params = [[p.detach().cpu().clone().requires_grad_(True) for p in n.parameters()] for n in nets]
    opt = FusedAdam([p for n in nets for p in n.parameters()], lr=5e-4)
    topt = torch.optim.Adam([p for ps in ref_params for p in ps], lr=5e-4)
    x = torch.rand(64, 3, device=DEV)
    d = torch.nn.functional.normalize(torch.randn(64, 3, device=DEV), dim=-1)
    g = torch.Generator().manual_seed(5)
    for step, scale in enumerate((3.0, 1e-3, 0.5), start=1):
        for n in nets:  # a forward packs (or re-uses) the images, as in training
            n(x, d if cfg.use_view_dirs else None)
        grads = [[torch.randn(p.shape, generator=g) * scale for p in ps] for ps in ref_params]
        for n, gs in zip(nets, grads):
            for p, gr in zip(n.parameters(), gs):
                p.grad = gr.to(DEV)
        for ps, gs in zip(ref_params, grads):
            for p, gr in zip(ps, gs):
                p.grad = gr.clone()
        allp = [p for n in nets for p in n.parameters()]
        targets = [n._fused_pack_target(n.flat_params()) for n in nets]
        assert all(t is not None for t in targets), "images current before the step: fused refresh expected"
        opt.step(clip_groups=[(allp, 1.0)])
        torch.nn.utils.clip_grad_norm_([p for ps in ref_params for p in ps], 1.0)
        topt.step()
        for n, ps in zip(nets, ref_params):
            got = n.flat_params().cpu()
            want = torch.cat([p.detach().reshape(-1) for p in ps])
            assert torch.allclose(got, want, rtol=2e-6, atol=1e-6), (name, step, (got - want).abs().max())
            # the images were refreshed in the Adam launch: no re-pack is pending ...
            assert n._packed_for_forward() is n._packed
            assert n._fused_pack_target(n.flat_params()) is not None
            # ... and they are exactly what nr_mlp_pack makes of the new parameters
            assert torch.equal(n._packed, _fresh_pack(n)), (name, step)


def test_pack_table_covers_every_parameter():
    """Every flat parameter but the two head biases (read from the fp32 parameters by
    the kernels) has at least one image destination, offsets lie inside the packed
    images, and no two parameters share a destination."""
    from noisy_src.config import ModelConfig
    from noisy_src.model import NeRF
    for prec in ("bf16", "fp32"):
        net = NeRF(ModelConfig(precision=prec)).to(DEV)
        net.flat_params()
        net._packed_for_forward()
        t = net._pack_table().cpu()
        n = net._param_count
        t = t.reshape(3, n).to(torch.int64) & 0xFFFFFFFF
        kind, off = t >> 29, t & ((1 << 29) - 1)
        has = (kind > 0).sum(0) >= 1
        off0, none = 0, []
        for pname, prm in net.named_parameters():
            if pname in ("sigma_linear.bias", "rgb_linear.bias"):
                none += list(range(off0, off0 + prm.numel()))
            off0 += prm.numel()
        expect = torch.ones(n, dtype=torch.bool)
        expect[none] = False
        assert torch.equal(has, expect), (prec, (has != expect).nonzero()[:10])
        used = off[kind > 0]
        assert int(used.max()) < net._packed.numel()
        assert used.unique().numel() == used.numel(), prec


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_trainer_fused_tail_equals_adam_then_repack(precision):
    """Full Trainer steps (coarse + fine in one clip group) with the fused tail vs the
    same steps with the images re-packed by the next forward instead: bit-identical
    parameters, losses and images (clip inactive, so both tails scale by exactly 1)."""
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import Trainer
    from noisy_src.model import create_nerf
    from noisy_src.optim import FusedAdam
    rc = RenderConfig(num_samples=32, num_samples_fine=32)
    trainers = []
    for refresh in (True, False):
        torch.manual_seed(7)
        mc, mf = create_nerf(ModelConfig(precision=precision))
        tr = Trainer(mc.to(DEV), mf.to(DEV), rc, max_norm=1e9)
        if not refresh:
            tr.optimizer = FusedAdam(tr.params, lr=5e-4, refresh_images=False)
            tr.scheduler = torch.optim.lr_scheduler.LambdaLR(tr.optimizer, tr.scheduler.lr_lambdas[0])
        trainers.append(tr)
    g = torch.Generator().manual_seed(9)
    B = 256
    for _ in range(3):
        o = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])
        dd = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0]), dim=-1)
        tgt = torch.rand(B, 3, generator=g)
        t_rand = torch.rand(B, rc.num_samples, generator=g).to(DEV)
        u = torch.rand(B, rc.num_samples_fine, generator=g).to(DEV)
        losses = [float(tr.step(o.to(DEV), dd.to(DEV), tgt.to(DEV), t_rand=t_rand, u=u)["loss"]) for tr in trainers]
        assert losses[0] == losses[1]
    a, b = trainers
    for na, nb in ((a.model_coarse, b.model_coarse), (a.model_fine, b.model_fine)):
        assert torch.equal(na.flat_params(), nb.flat_params())
        assert torch.equal(na._packed, _fresh_pack(na))
        assert torch.equal(nb._packed_for_forward(), _fresh_pack(nb))
    # both took the whole-network fast path (flat buffers straight from the networks)
    for tr in trainers:
        plans = list(tr.optimizer._nerf_plans.values())
        assert plans and all(plans) and len(plans[0]) == 2
        # the step consumed the flat gradients and dropped the networks' extra reference
        # to them, so zero_grad(set_to_none=True) frees them
        assert tr.model_coarse._last_gflat is None and tr.model_fine._last_gflat is None


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_graphed_trainer_equals_eager_trainer(precision):
    """engine.GraphedTrainer (the step captured once into a hipGraph and replayed, the
    Adam schedule advanced through its device pair) performs exactly the eager
    Trainer's steps: bit-identical losses, parameters, packed images, LR and Adam step
    counters, with the randoms injected through the static inputs."""
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import GraphedTrainer, Trainer
    from noisy_src.model import create_nerf
    rc = RenderConfig(num_samples=32, num_samples_fine=32)
    trainers = []
    for _ in range(2):
        torch.manual_seed(17)
        mc, mf = create_nerf(ModelConfig(precision=precision))
        trainers.append(Trainer(mc.to(DEV), mf.to(DEV), rc))
    eager, tr_g = trainers
    g = torch.Generator().manual_seed(23)
    B = 256

    def batch():
        o = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])
        dd = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0]), dim=-1)
        return [t.to(DEV) for t in (o, dd, torch.rand(B, 3, generator=g), torch.rand(B, rc.num_samples, generator=g),
                                    torch.rand(B, rc.num_samples_fine, generator=g))]

    b0 = batch()
    graphed = GraphedTrainer(tr_g, *b0, warmup=2)
    for _ in range(2):
        eager.step(*b0)
    for k in range(5):
        bk = batch()
        le = float(eager.step(*bk)["loss"])
        lg = float(graphed.step(*bk)["loss"])
        assert le == lg, (k, le, lg)
    for na, nb in ((eager.model_coarse, tr_g.model_coarse), (eager.model_fine, tr_g.model_fine)):
        assert torch.equal(na.flat_params(), nb.flat_params())
        assert torch.equal(nb._packed, _fresh_pack(nb))
    assert eager.optimizer.param_groups[0]["lr"] == tr_g.optimizer.param_groups[0]["lr"]
    pe, pg = eager.params[0], tr_g.params[0]
    assert int(eager.optimizer.state[pe]["step"]) == int(tr_g.optimizer.state[pg]["step"]) == 7


def test_graphed_trainer_draws_the_eager_randoms():
    """Without injected randoms, GraphedTrainer draws the jitter and inverse-CDF uniforms
    with torch.rand into its static buffers before each replay (no RNG inside the graph):
    the same draws, in the same order, as the eager Trainer's own torch.rand calls, so
    from the same seed both train bit-identically (coarse stream on: 512 rays)."""
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import GraphedTrainer, Trainer
    from noisy_src.model import create_nerf
    rc = RenderConfig(num_samples=32, num_samples_fine=64)
    trainers = []
    for _ in range(2):
        torch.manual_seed(5)
        mc, mf = create_nerf(ModelConfig(precision="bf16"))
        trainers.append(Trainer(mc.to(DEV), mf.to(DEV), rc, coarse_stream="auto"))
    eager, tr_g = trainers
    g = torch.Generator().manual_seed(29)
    B = 512
    o = (torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])).to(DEV)
    dd = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0]),
                                       dim=-1).to(DEV)
    tgt = torch.rand(B, 3, generator=g).to(DEV)
    torch.manual_seed(77)
    le = [float(eager.step(o, dd, tgt)["loss"]) for _ in range(6)]
    torch.manual_seed(77)
    graphed = GraphedTrainer(tr_g, o, dd, tgt, warmup=2)
    assert tr_g.last_step_coarse_stream
    lg = [float(graphed.step()["loss"]) for _ in range(4)]  # steps 3-6 (the warm-ups were 1-2)
    assert le[2:] == lg, (le, lg)
    for na, nb in ((eager.model_coarse, tr_g.model_coarse), (eager.model_fine, tr_g.model_fine)):
        assert torch.equal(na.flat_params(), nb.flat_params())
