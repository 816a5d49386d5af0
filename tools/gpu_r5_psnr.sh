#!/bin/bash
# Round 5: more paired seeds of the reference-schedule PSNR comparison (lr_decay = 250):
# seeds FIRST .. FIRST+15, 8 worker processes sharing the GPU.  Usage: gpu_r5_psnr.sh FIRST
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
first=${1:-16}
timeout -k 10 1080 python -u tests/psnr_parity.py 2000 64 16 gpurun_out/r05_psnr_d250_s$first.json 250 8 $first > gpurun_out/r05_psnr_d250_s$first.log 2>&1
rc=$?; tail -4 gpurun_out/r05_psnr_d250_s$first.log; exit $rc
