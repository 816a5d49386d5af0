#!/bin/bash
# A/B on the GPU: tools/fwd_ab.py with a variant library (arg 1) vs the default build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
V=${1:-old}
NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$V timeout -k 10 240 python tools/fwd_ab.py save gpurun_out/ab_$V.pt > gpurun_out/ab_$V.log 2>&1 || { tail -20 gpurun_out/ab_$V.log; exit 1; }
cat gpurun_out/ab_$V.log
timeout -k 10 240 python tools/fwd_ab.py save gpurun_out/ab_new.pt > gpurun_out/ab_new.log 2>&1 || { tail -20 gpurun_out/ab_new.log; exit 1; }
cat gpurun_out/ab_new.log
python tools/fwd_ab.py compare gpurun_out/ab_$V.pt gpurun_out/ab_new.pt
