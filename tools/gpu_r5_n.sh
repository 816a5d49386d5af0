#!/bin/bash
# Round 5: kernel trace of the 512-ray graph replay (coarse chain as a second branch).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_b512g
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_b512g -o run --output-format csv -- python bench.py --batch 512 --graph --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_b512g.log 2>&1 || { tail -n 20 gpurun_out/prof_b512g.log; exit 3; }
ls gpurun_out/prof_b512g
