#!/bin/bash
# GPU-box A/B of kernel-variant libraries: for each variant, the -m gpu parity
# tests against it (NR_HIP_LIB), then the fused-MLP microbench.  The default
# build's microbench runs first for reference.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/mb_default.log 2>&1 || { tail -20 gpurun_out/mb_default.log; exit 3; }
echo "== default"; grep bf16 gpurun_out/mb_default.log
for v in "$@"; do
  if [ "$v" = default ]; then export NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/libnerf_hip.so; else export NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v; fi
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1
  rc=$?; echo "== $v pytest rc=$rc"; tail -3 gpurun_out/pytest_$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/mb_$v.log 2>&1 || { tail -20 gpurun_out/mb_$v.log; exit 4; }
  grep bf16 gpurun_out/mb_$v.log
done
