#!/bin/bash
# Refresh every round-5 bench record on the final tree (one box, one session): the
# BASELINE configs beside the default line, each bench run under its own time limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/rec
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/rec/r05_bench_$n.json 2> gpurun_out/rec/r05_bench_$n.err
  local r=$?
  if [ $r -ne 0 ]; then echo "bench $n rc=$r"; tail -20 gpurun_out/rec/r05_bench_$n.err; exit 5; fi
  python -c "import json;d=json.load(open('gpurun_out/rec/r05_bench_$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
run default --steps 200 --warmup 20 --no-cpu-baseline
run b512_graph --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run dp_b512_graph --dp --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run dp_b512 --dp --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline
run pose_opt --pose-opt --steps 20 --warmup 5 --no-cpu-baseline
run cfg5_fp16 --precision fp16 --num-samples 128 --num-samples-fine 256 --steps 20 --warmup 5 --no-cpu-baseline
run fp32 --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline
run eval --eval
