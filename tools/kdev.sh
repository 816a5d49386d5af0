#!/bin/bash
# Fast inspection build of csrc/mlp.hip (default model instances only):
# per-kernel registers/spills, and the gfx950 ISA in /tmp/mlp_dev.s.
set -e
SRC=/root/repo/robust-nerf_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off \
  -DNR_MLP_DEV -I/root/repo/include -I$SRC -c $SRC/mlp.hip -o /tmp/mlp_dev.o "$@"
/root/repo/tools/kres.sh /tmp/mlp_dev.o
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off -DNR_MLP_DEV \
  -I/root/repo/include -I$SRC --cuda-device-only -S $SRC/mlp.hip -o /tmp/mlp_dev.s "$@"
