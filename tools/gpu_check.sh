#!/bin/bash
# GPU-box check: parity tests (no -x: collect every failure), then the fused-MLP
# microbench for the default build and any variant libraries given as args.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/microbench_mlp.py bf16 fp32 > gpurun_out/mb_default.log 2>&1 || { cat gpurun_out/mb_default.log | tail -20; exit 3; }
cat gpurun_out/mb_default.log
for v in "$@"; do
  NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/mb_$v.log 2>&1 || { tail -20 gpurun_out/mb_$v.log; exit 4; }
  echo "== $v"; cat gpurun_out/mb_$v.log
done
exit $rc
