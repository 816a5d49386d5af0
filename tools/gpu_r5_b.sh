#!/bin/bash
# Round 5: the 8-wave layer-pipelined backward (v2) -- bit-identity tests, then the
# fused-vs-split microbench and a same-box step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pipe.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r5b_pipe.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r5b_pipe.log | tail -25; [ $rc = 0 ] || exit 2
MB_KERNELS=bwd_dx,bwd_dw,bwd_dxdw,bwd_dx,bwd_dw,bwd_dxdw timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/r5b_mb.log 2>&1 || { tail -20 gpurun_out/r5b_mb.log; exit 3; }
grep -E "^bf16" gpurun_out/r5b_mb.log
MB_M=262144 MB_KERNELS=bwd_dx,bwd_dw,bwd_dxdw timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/r5b_mb_c.log 2>&1 || { tail -20 gpurun_out/r5b_mb_c.log; exit 4; }
grep -E "^bf16" gpurun_out/r5b_mb_c.log
for mode in split fused split fused; do
  NR_MLP_BACKWARD=$mode timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r5b_bench_$mode.json 2> gpurun_out/r5b_bench_$mode.err || { tail -20 gpurun_out/r5b_bench_$mode.err; exit 5; }
  python -c "import json;d=json.load(open('gpurun_out/r5b_bench_$mode.json'));print('$mode', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
