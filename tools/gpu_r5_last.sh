#!/bin/bash
# Round-5 last session: the full GPU suite on the final tree, tools/gpu_profile.sh (smoke,
# default bench, rocprofv3 kernel trace, HBM PMC passes), and a kernel trace of the cfg #5
# (fp16, 128c+256f) step for the record.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/cfg5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05_last_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r05_last_pytest.log; [ $rc = 0 ] || exit 2
bash tools/gpu_profile.sh || exit 3
rm -rf gpurun_out/cfg5/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg5/prof -o run --output-format csv -- python bench.py --precision fp16 --num-samples 128 --num-samples-fine 256 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/cfg5/prof.log 2>&1 || { tail -n 20 gpurun_out/cfg5/prof.log; exit 4; }
ls gpurun_out/cfg5/prof
