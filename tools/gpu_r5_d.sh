#!/bin/bash
# Round 5: 8-wave pipeline with the dir stage's heads work moved off its critical path --
# bit-identity tests, microbench (fine / coarse M) and the per-stage in-kernel timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pipe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r5d_pipe.log 2>&1
rc=$?; tail -3 gpurun_out/r5d_pipe.log; [ $rc = 0 ] || exit 2
for M in 786432 262144; do
  MB_M=$M MB_KERNELS=bwd_dx,bwd_dw,bwd_dxdw,bwd_dxdw timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/r5d_mb_$M.log 2>&1 || { tail -20 gpurun_out/r5d_mb_$M.log; exit 3; }
  grep -E "^bf16" gpurun_out/r5d_mb_$M.log
done
NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/pipeprof timeout -k 10 200 python tools/pipe_prof.py > gpurun_out/r5d_pipeprof.log 2>&1 || { tail -20 gpurun_out/r5d_pipeprof.log; exit 4; }
cat gpurun_out/r5d_pipeprof.log
