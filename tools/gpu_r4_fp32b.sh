#!/bin/bash
# fp32 forward read-ahead + scratch fixes: the whole -m gpu suite, smoke, then the cfg #2
# fp32 and default bench lines.  Any failure ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
bash tools/gpu_r4_tests.sh || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04_fp32_bench.json 2> gpurun_out/r04_fp32_bench.err || { tail -20 gpurun_out/r04_fp32_bench.err; exit 2; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_default_bench.json 2> gpurun_out/r04_default_bench.err || { tail -20 gpurun_out/r04_default_bench.err; exit 3; }
python -c "
import json
for f in ['r04_fp32_bench','r04_default_bench']:
    d=json.load(open('gpurun_out/'+f+'.json'));print(f, d['value'], d['ms_per_step'], d['kernel_ms'])"
