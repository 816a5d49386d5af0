#!/bin/bash
# Fused-MLP microbench (bf16) for the default library and each named variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/mb_default.log 2>&1 || { tail -20 gpurun_out/mb_default.log; exit 3; }
echo "== default"; grep bf16 gpurun_out/mb_default.log
for v in "$@"; do
  NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/mb_$v.log 2>&1 || { tail -20 gpurun_out/mb_$v.log; exit 4; }
  echo "== $v"; grep bf16 gpurun_out/mb_$v.log
done
