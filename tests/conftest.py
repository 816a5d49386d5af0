"""pytest configuration: puts the package root on sys.path and registers markers.

`-m gpu` tests need a ROCm device (MI355X) and the built HIP library; the
`-m "not gpu"` suite covers the oracle, host logic and the library's exports.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "robust-nerf_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: longer-running test")
