#!/usr/bin/env python3
"""How many 32-sample MLP tiles carry a nonzero incoming gradient.

A sample whose sigma is exactly 0 (alpha = w = 0, and torch's ReLU'(0) = 0 zeroes
d sigma: reference rendering.py:83) or whose transmittance has underflowed to 0
(cumprod of 1 - alpha + 1e-10, rendering.py:87-96) gets exactly zero g_rgb and
g_sigma from the compositing backward, so every layer's dz for it is zero.  This
tool counts, per network, the fraction of 32-sample tiles with ANY nonzero
g_rgb / g_sigma entry, as the HIP composite backward produced them:

* ``bench``: bench.py's cfg #2 step (seed-42 init, lego cameras, random targets),
  at the first step and after ``--steps`` steps;
* ``trained``: tests/psnr_parity.py's analytic 3-sphere scene (lego training
  cameras), trained by engine.Trainer for ``--iters`` iterations at 1024 rays,
  then measured on 4096-ray batches of its training rays.

    python tools/active_tiles.py [--iters 2000] [--steps 20] [--out gpurun_out/active_tiles.json]
"""

from __future__ import annotations

import argparse
import json
import math
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "robust-nerf_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

SPHERES = [((0.0, 0.0, 0.0), 0.7, (0.9, 0.2, 0.1)), ((0.8, 0.3, 0.2), 0.35, (0.1, 0.7, 0.2)),
           ((-0.5, -0.6, 0.4), 0.45, (0.2, 0.3, 0.9))]


def scene_field(pts):
    """tests/psnr_parity.py's analytic field (soft-edged coloured spheres)."""
    sigma = torch.zeros(pts.shape[:-1], device=pts.device)
    rgb = torch.ones(*pts.shape[:-1], 3, device=pts.device)
    for c, r, col in SPHERES:
        d = (pts - torch.tensor(c, device=pts.device)).norm(dim=-1)
        s = 40.0 * torch.sigmoid((r - d) * 40.0)
        w = (s / (sigma + s + 1e-6))[..., None]
        rgb = rgb * (1 - w) + torch.tensor(col, device=pts.device) * w
        sigma = sigma + s
    return rgb, sigma


def scene_rays(size: int, dev):
    """Every pixel ray of the 100 lego training cameras at size x size, and the analytic
    scene's ground truth rendered with the HIP sampler / compositor (256 samples)."""
    from noisy_src import ops
    from noisy_src.rays import get_ray_directions, get_rays
    fix = sorted((ROOT / "tests" / "golden").glob("final_poses_*.npz"))[0]
    poses = torch.from_numpy(np.load(fix)["ground_truth_poses"]).float().to(dev)
    focal = 0.5 * size / math.tan(0.5 * 0.6911112070083618)
    dirs = get_ray_directions(size, size, focal).to(dev)
    o, d = zip(*[get_rays(dirs, p) for p in poses])
    o, d = torch.stack(o).reshape(-1, 3), torch.stack(d).reshape(-1, 3)
    with torch.no_grad():
        pts, z = ops.stratified_sample(o, d, 2.0, 6.0, 256)
        rgb, sigma = scene_field(pts)
        gt = ops.composite(rgb.contiguous(), sigma.contiguous(), z, d)[0]
    return o, d, gt


class Probe:
    """Wraps the fused MLP's backward: per call, tiles with a nonzero incoming gradient."""

    def __init__(self):
        self.rec = []
        self.on = False

    def install(self):
        from noisy_src import model
        orig = model._MLPFunction.backward
        probe = self

        def backward(ctx, g_rgb, g_sigma):
            if probe.on and g_rgb is not None and g_sigma is not None:
                M = g_rgb.shape[0]
                nz = (g_rgb != 0).any(-1) | (g_sigma.reshape(-1) != 0)
                pad = (-M) % 32
                t = torch.nn.functional.pad(nz, (0, pad)).reshape(-1, 32)
                probe.rec.append({"M": M, "tiles": t.shape[0], "active_tiles": int(t.any(-1).sum()),
                                  "active_samples": int(nz.sum())})
            return orig(ctx, g_rgb, g_sigma)

        model._MLPFunction.backward = staticmethod(backward)

    def take(self):
        out, self.rec = self.rec, []
        by_m = {}
        for r in out:
            a = by_m.setdefault(r["M"], {"M": r["M"], "calls": 0, "tiles": 0, "active_tiles": 0, "active_samples": 0})
            a["calls"] += 1
            for k in ("tiles", "active_tiles", "active_samples"):
                a[k] += r[k]
        for a in by_m.values():
            a["active_tile_frac"] = round(a["active_tiles"] / a["tiles"], 4)
            a["active_sample_frac"] = round(a["active_samples"] / (a["M"] * a["calls"]), 4)
        return sorted(by_m.values(), key=lambda a: a["M"])


def bench_state(probe, steps: int, dev):
    import bench
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import Trainer
    from noisy_src.model import create_nerf
    torch.manual_seed(42)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    tr = Trainer(mc.to(dev), mf.to(dev), RenderConfig())
    pool = [bench.lego_rays(4096, k, dev) for k in range(4)]
    torch.manual_seed(1234)
    out = {}
    probe.on = True
    tr.step(*pool[0])
    out["step0"] = probe.take()
    probe.on = False
    for k in range(1, steps):
        tr.step(*pool[k % 4])
    probe.on = True
    for k in range(4):
        tr.step(*pool[k])
    out[f"steps{steps}_to_{steps + 4}"] = probe.take()
    probe.on = False
    return out


def trained_state(probe, iters: int, size: int, dev):
    from noisy_src.config import ModelConfig, RenderConfig
    from noisy_src.engine import Trainer
    from noisy_src.model import create_nerf
    o, d, gt = scene_rays(size, dev)
    n_train = 90 * size * size
    torch.manual_seed(42)
    mc, mf = create_nerf(ModelConfig(precision="bf16"))
    tr = Trainer(mc.to(dev), mf.to(dev), RenderConfig())
    g = torch.Generator(device=dev).manual_seed(0)
    out = {}
    t0 = time.time()
    marks = sorted({0, 500, 1000, iters})
    for it in range(iters + 1):
        measure = it in marks
        if measure:
            probe.on = True
            for _ in range(4):
                idx = torch.randint(0, n_train, (4096,), device=dev, generator=g)
                tr.step(o[idx], d[idx], gt[idx])
            out[f"iter{it}"] = probe.take()
            probe.on = False
            print(f"iter {it}: {out[f'iter{it}']} ({time.time() - t0:.1f} s)", flush=True)
        if it == iters:
            break
        idx = torch.randint(0, n_train, (1024,), device=dev, generator=g)
        tr.step(o[idx], d[idx], gt[idx])
    # test-view PSNR of the trained state (deterministic renders of views 90..99)
    from noisy_src.rendering import render_rays
    with torch.no_grad():
        ps = []
        for v in range(90, 100):
            sl = slice(v * size * size, (v + 1) * size * size)
            rgb = render_rays(mc, mf, o[sl], d[sl], RenderConfig(), is_train=False)["rgb_fine"]
            ps.append(-10 * math.log10(float(torch.mean((rgb - gt[sl]) ** 2))))
    out["test_psnr_db"] = round(float(np.mean(ps)), 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/active_tiles.json")
    args = ap.parse_args()
    dev = torch.device("cuda")
    probe = Probe()
    probe.install()
    rec = {"tool": "tools/active_tiles.py", "tile": 32,
           "bench_cfg2": bench_state(probe, args.steps, dev)}
    print(json.dumps(rec["bench_cfg2"]), flush=True)
    rec["trained_3sphere"] = trained_state(probe, args.iters, args.size, dev)
    rec["trained_3sphere"].update({"iters": args.iters, "size": args.size, "train_batch": 1024,
                                   "measure_batch": 4096})
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(rec, indent=1))
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
