#!/bin/bash
# GPU: the -m gpu suite (stop at the first failure), then the fused-MLP microbench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python tools/microbench_mlp.py bf16 > gpurun_out/mb_default.log 2>&1 || { tail -20 gpurun_out/mb_default.log; exit 3; }
grep bf16 gpurun_out/mb_default.log
