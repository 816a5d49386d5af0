#!/bin/bash
# Build an A/B variant of libnerf_hip.so with extra -D flags on mlp.hip only:
#   tools/build_variant.sh NAME -DFLAG=V ...   -> noisy_src/lib/variants/NAME
# (the other objects come from the default build in robust-nerf_amd/build/).
set -e
NAME=$1; shift
R=/root/repo/robust-nerf_amd
mkdir -p $R/build/var_$NAME $R/noisy_src/lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=off \
  -Wno-unused-function -I/root/repo/include -I$R/csrc -DNR_AB_VARIANT "$@" -c $R/csrc/mlp.hip -o $R/build/var_$NAME/mlp.o
OBJS=$(ls $R/build/*.o | grep -v "/mlp.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $R/build/var_$NAME/mlp.o -o $R/noisy_src/lib/variants/$NAME
echo built $R/noisy_src/lib/variants/$NAME
