#!/bin/bash
# Round 5: what bounds the 8-wave pipeline -- timing-only variants without the dz ring
# traffic / the activation staging / both, and the per-stage in-kernel timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default noring nostage neither; do
  lib=""; [ $v = default ] || lib=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v
  for M in 786432 262144; do
    NR_HIP_LIB=$lib MB_M=$M MB_KERNELS=bwd_dxdw,bwd_dxdw,bwd_dxdw timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/r5c_$v_$M.log 2>&1 || { tail -20 gpurun_out/r5c_$v_$M.log; exit 3; }
    echo "== $v"; grep -E "^bf16" gpurun_out/r5c_$v_$M.log
  done
done
NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/pipeprof timeout -k 10 200 python tools/pipe_prof.py > gpurun_out/r5c_pipeprof.log 2>&1 || { tail -20 gpurun_out/r5c_pipeprof.log; exit 4; }
cat gpurun_out/r5c_pipeprof.log
