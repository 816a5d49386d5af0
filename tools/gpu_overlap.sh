#!/bin/bash
# Backward-chain stream-overlap A/B (tools/microbench_overlap.py), then the dW variant microbench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/microbench_overlap.py > gpurun_out/mb_overlap.log 2>&1 || { tail -20 gpurun_out/mb_overlap.log; exit 3; }
grep overlap gpurun_out/mb_overlap.log
bash tools/gpu_mb.sh "$@"
