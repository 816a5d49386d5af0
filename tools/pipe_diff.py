"""Where do the fused and split backward differ?  Per parameter tensor mismatch counts
for a few sample counts (diagnostic; uses tests/test_pipe.py's runner)."""

import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "robust-nerf_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_pipe import _net, _run  # noqa: E402


def main():
    net = _net("bf16")
    names = [(n, p.numel()) for n, p in net.named_parameters()]
    for M in [int(v) for v in (sys.argv[1:] or ["100", "1000", "4000", "12807"])]:
        (g0, _, _, _), (g1, _, _, status) = _run(net, M)
        bad = (g0 != g1)
        print(f"M={M}: status {status}, {int(bad.sum())} of {g0.numel()} differ")
        off = 0
        for n, c in names:
            b = int(bad[off:off + c].sum())
            if b:
                d = (g0[off:off + c] - g1[off:off + c]).abs().max().item()
                print(f"   {n:40s} {b:7d}/{c:7d}  max {d:.3e}  ref max {g0[off:off + c].abs().max().item():.3e}")
            off += c


if __name__ == "__main__":
    main()
