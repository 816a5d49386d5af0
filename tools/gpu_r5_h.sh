#!/bin/bash
# Round 5: layer-pipelined backward, hand-off signals stored after the dX product
# (NR_PIPE_LATE_SIG=1) vs right after the barrier: pipe parity on the variant, per-stage
# timing of both, and the fused backward in isolation, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/robust-nerf_amd/noisy_src/lib/variants
NR_HIP_LIB=$V/late timeout -k 10 300 python -u -m pytest tests/test_pipe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r5h_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r5h_pytest.log; [ $rc = 0 ] || exit 2
for v in pipeprof pipeprof_late; do
  NR_HIP_LIB=$V/$v timeout -k 10 200 python tools/pipe_prof.py > gpurun_out/r5h_$v.log 2>&1 || { tail -n 20 gpurun_out/r5h_$v.log; exit 3; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r5h_$v.log
done
for i in 1 2; do
  for v in default late; do
    lib=""; [ $v = default ] || lib=$V/$v
    for M in 786432 262144; do
      NR_HIP_LIB=$lib MB_M=$M MB_REPS=5 MB_KERNELS=bwd_dxdw,bwd_dxdw timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/r5h_mb_${v}_${M}_$i.log 2>&1 || { tail -n 20 gpurun_out/r5h_mb_${v}_${M}_$i.log; exit 4; }
      echo "== $v $M $i"; grep -E "^bf16" gpurun_out/r5h_mb_${v}_${M}_$i.log
    done
  done
done
