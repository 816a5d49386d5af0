"""Training-loop throughput of the three ways the CLI (noisy_src.train) can drive a step,
at B rays on one GPU (bf16, cfg #2 shape):
  sync   -- trainer.step, then the logged losses read back at once (.tolist(): the
            reference's per-iteration .item() pattern, train.py:386-420)
  lagged -- trainer.step, losses read back one iteration late (engine.LaggedScalars,
            what train.train now does)
  graph  -- GraphedTrainer replay + lagged readback (train --graph)
Each mode draws t_rand / u per step on the host stream as train.train does.
python tools/cli_loop.py [B ...]   (default 1024 4096); prints one JSON line per (B, mode)."""
import json
import sys
import time

import torch

sys.path[:0] = [".", "robust-nerf_amd"]
import bench  # noqa: E402
from noisy_src.config import ModelConfig, RenderConfig  # noqa: E402
from noisy_src.engine import GraphedTrainer, LaggedScalars, Trainer, mean_over_ranks  # noqa: E402
from noisy_src.model import create_nerf  # noqa: E402

K, WARM = 100, 10
dev = torch.device("cuda", 0)
rc = RenderConfig()


def run(B, mode):
    torch.manual_seed(42)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    tr = Trainer(mc.to(dev), mf.to(dev), rc)
    pool = [bench.lego_rays(B, k, dev) for k in range(4)]

    def draws():
        return torch.rand(B, rc.num_samples, device=dev), torch.rand(B, rc.num_samples_fine, device=dev)

    tr.step(*pool[0][:3], *draws())
    g = GraphedTrainer(tr, *pool[1][:3], *draws(), warmup=0) if mode == "graph" else None
    lag = LaggedScalars()
    for k in range(WARM + K):
        if k == WARM:
            lag.flush()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        batch = pool[k % 4][:3]
        m = g.step(*batch, *draws()) if g is not None else tr.step(*batch, *draws())
        vals = mean_over_ranks([m["loss"], m["loss_coarse"], m["loss_fine"]])
        if mode == "sync":
            vals.tolist()
        else:
            lag.push(vals)
    lag.flush()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    return {"B": B, "mode": mode, "ms_per_step": round(1e3 * dt, 4), "rays_per_s": round(B / dt)}


for B in [int(a) for a in sys.argv[1:]] or [1024, 4096]:
    for mode in ("sync", "lagged", "graph"):
        print(json.dumps(run(B, mode)), flush=True)
