"""Host-side (Python) cost of one eager training step at a small batch: cProfile over
K steps of engine.Trainer at B rays (GPU).  python tools/prof_host.py [B] [K]"""
import cProfile
import pstats
import sys
import time

import torch

sys.path[:0] = [".", "robust-nerf_amd"]
import bench  # noqa: E402
from noisy_src.config import ModelConfig, RenderConfig  # noqa: E402
from noisy_src.engine import Trainer  # noqa: E402
from noisy_src.model import create_nerf  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda", 0)
torch.manual_seed(42)
mc, mf = create_nerf(ModelConfig(precision="bf16"))
tr = Trainer(mc.to(dev), mf.to(dev), RenderConfig())
pool = [bench.lego_rays(B, k, dev) for k in range(4)]
for k in range(10):
    tr.step(*pool[k % 4])
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    tr.step(*pool[k % 4])
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"B={B}: host issue {1e3 * t_host / K:.3f} ms/step, wall {1e3 * t_all / K:.3f} ms/step")
pr = cProfile.Profile()
pr.enable()
for k in range(K):
    tr.step(*pool[k % 4])
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(30)
