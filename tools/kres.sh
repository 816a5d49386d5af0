#!/bin/bash
# Per-kernel register / spill / LDS usage of a built HIP object (default: build/mlp.o).
set -e
OBJ=${1:-/root/repo/robust-nerf_amd/build/mlp.o}
TMP=$(mktemp -d)
cp "$OBJ" "$TMP/k.o"
cd "$TMP"
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o > /dev/null
/opt/rocm/lib/llvm/bin/llvm-readelf --notes k.o.0.hipv4-amdgcn-amd-amdhsa--gfx950 |
  grep -E "^\s+\.name:|\.vgpr_count|\.agpr_count|spill_count|group_segment_fixed_size" | grep -v args |
  sed 's/  */ /g' | paste -d' ' - - - - - - | sed 's/_ZN2nr//' | cut -c1-220
rm -rf "$TMP"
