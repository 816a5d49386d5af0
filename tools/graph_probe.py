"""Capture check of engine.GraphedTrainer for one configuration: E eager Trainer steps,
then GraphedTrainer(warmup=W) on B rays, then 3 replays against an eager twin.
python tools/graph_probe.py B W E [num_samples num_samples_fine]"""
import sys

import torch

sys.path[:0] = [".", "robust-nerf_amd"]
from noisy_src.config import ModelConfig, RenderConfig  # noqa: E402
from noisy_src.engine import GraphedTrainer, Trainer  # noqa: E402
from noisy_src.model import create_nerf  # noqa: E402

B, W, E = (int(a) for a in sys.argv[1:4])
ns, nf = (int(a) for a in sys.argv[4:6]) if len(sys.argv) > 5 else (64, 128)
dev = torch.device("cuda", 0)
rc = RenderConfig(num_samples=ns, num_samples_fine=nf)
g = torch.Generator().manual_seed(5)


def batch():
    o = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 4.0])
    d = torch.nn.functional.normalize(torch.randn(B, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0]), dim=-1)
    return [t.to(dev) for t in (o, d, torch.rand(B, 3, generator=g), torch.rand(B, ns, generator=g),
                                torch.rand(B, nf, generator=g))]


trs = []
for _ in range(2):
    torch.manual_seed(3)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    trs.append(Trainer(mc.to(dev), mf.to(dev), rc))
eager, tg = trs
pre = [batch() for _ in range(E)]
for b in pre:
    eager.step(*b)
    tg.step(*b)
b0 = batch()
print(f"B={B} W={W} E={E}: capturing", flush=True)
gr = GraphedTrainer(tg, *b0, warmup=W)
torch.cuda.synchronize()
print("captured", flush=True)
for _ in range(W):
    eager.step(*b0)
for k in range(3):
    bk = batch()
    le, lg = float(eager.step(*bk)["loss"]), float(gr.step(*bk)["loss"])
    print(k, le, lg, flush=True)
    assert le == lg
print("ok", flush=True)
