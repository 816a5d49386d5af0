"""GPU: the coarse network's chain on its own stream (engine.Trainer(coarse_stream=True),
VERDICT r4 item 3).  The coarse forward, compositing and -- through autograd's stream
semantics -- their backward run beside the fine network's (the chains are independent:
reference rays.py:325 detaches the fine samples), eagerly and as two branches of a
GraphedTrainer capture.  Same kernels on the same inputs: losses, parameters and Adam
state must be BIT-identical to the one-stream step."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(precision="bf16", ns=64, nf=128):
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import Trainer
    from noisy_src.model import create_nerf
    rc = RenderConfig(num_samples=ns, num_samples_fine=nf)
    out = []
    for cs in (False, True):
        torch.manual_seed(17)
        mc, mf = create_nerf(ModelConfig(precision=precision))
        out.append(Trainer(mc.to(DEV), mf.to(DEV), rc, coarse_stream=cs))
    return rc, out


def _batches(rc, B, n, seed=23):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        o = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])
        d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0]), dim=-1)
        out.append([t.to(DEV) for t in (o, d, torch.rand(B, 3, generator=g),
                                         torch.rand(B, rc.num_samples, generator=g),
                                         torch.rand(B, rc.num_samples_fine, generator=g))])
    return out


def _same(a, b):
    for na, nb in ((a.model_coarse, b.model_coarse), (a.model_fine, b.model_fine)):
        assert torch.equal(na.flat_params(), nb.flat_params())
    sa, sb = list(a.optimizer._flat_state.values()), list(b.optimizer._flat_state.values())
    assert len(sa) == len(sb) > 0
    for (ma, va), (mb, vb) in zip(sa, sb):
        assert torch.equal(ma, mb) and torch.equal(va, vb)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_coarse_stream_eager_equals_one_stream(precision):
    rc, (one, two) = _pair(precision, 32, 64)
    for k, b in enumerate(_batches(rc, 512, 4)):
        l1 = float(one.step(*b)["loss"])
        l2 = float(two.step(*b)["loss"])
        assert l1 == l2, (k, l1, l2)
    _same(one, two)


def test_coarse_stream_graph_equals_eager():
    """cfg #4's per-rank size (512 rays, 64c+128f): the two-branch graph replay equals the
    one-stream eager step bit for bit."""
    from noisy_src.engine import GraphedTrainer
    rc, (one, two) = _pair("bf16")
    bs = _batches(rc, 512, 7)
    graphed = GraphedTrainer(two, *bs[0], warmup=2)
    for _ in range(2):
        one.step(*bs[0])
    for k, b in enumerate(bs[1:]):
        le = float(one.step(*b)["loss"])
        lg = float(graphed.step(*b)["loss"])
        assert le == lg, (k, le, lg)
    _same(one, two)


def test_auto_engages_only_in_small_graph_replays():
    """coarse_stream="auto" (bench.py / train.py default): eager steps stay on one stream;
    a GraphedTrainer capture of <= AUTO_COARSE_STREAM_RAYS rays gets the second branch,
    and its replays equal the one-stream eager step bit for bit."""
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import GraphedTrainer, Trainer
    from noisy_src.model import create_nerf
    rc = RenderConfig(num_samples=64, num_samples_fine=128)
    torch.manual_seed(17)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    one = Trainer(mc.to(DEV), mf.to(DEV), rc, coarse_stream=False)
    torch.manual_seed(17)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    auto = Trainer(mc.to(DEV), mf.to(DEV), rc, coarse_stream="auto")
    bs = _batches(rc, 512, 5)
    assert 512 <= Trainer.AUTO_COARSE_STREAM_RAYS
    auto.step(*bs[0])
    assert not auto.last_step_coarse_stream  # eager: one stream
    one.step(*bs[0])
    graphed = GraphedTrainer(auto, *bs[1], warmup=1)
    one.step(*bs[1])
    assert auto.last_step_coarse_stream  # the capture took the two-branch form
    for k, b in enumerate(bs[2:]):
        le = float(one.step(*b)["loss"])
        lg = float(graphed.step(*b)["loss"])
        assert le == lg, (k, le, lg)
    _same(one, auto)


def test_coarse_stream_rejects_unknown_mode():
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import Trainer
    from noisy_src.model import create_nerf
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    with pytest.raises(ValueError, match="coarse_stream"):
        Trainer(mc, mf, RenderConfig(), coarse_stream="sometimes")
