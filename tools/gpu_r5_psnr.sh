#!/bin/bash
# Round 5: more paired seeds of the reference-schedule PSNR comparison (lr_decay = 250).
# Usage: gpu_r5_psnr.sh FIRST [N_SEEDS [WORKERS]]  (default 16 seeds, 8 worker processes
# sharing the GPU: seeds FIRST .. FIRST+N-1)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
first=${1:-16}; n=${2:-16}; w=${3:-8}
timeout -k 10 1080 python -u tests/psnr_parity.py 2000 64 $n gpurun_out/r05_psnr_d250_s$first.json 250 $w $first > gpurun_out/r05_psnr_d250_s$first.log 2>&1
rc=$?; tail -n 4 gpurun_out/r05_psnr_d250_s$first.log; exit $rc
