#!/bin/bash
# Round 5: the data-parallel all-reduce timing moved out of the timed region -- the eager
# 512-ray DP step against the plain eager 512-ray step, and the world-1 4096-ray DP line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/rec
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/rec/r05_bench_$n.json 2> gpurun_out/rec/r05_bench_$n.err || { tail -n 20 gpurun_out/rec/r05_bench_$n.err; exit 5; }
  python -c "import json;d=json.load(open('gpurun_out/rec/r05_bench_$n.json'));t=d.get('topology');print('$n', d['value'], d['ms_per_step'], t and [(r['allreduce_span_ms'] if 'allreduce_span_ms' in r else None, r.get('allreduce_exposed_ms')) for r in t['ranks']])"
}
for i in 1 2; do
  run dp_b512 --dp --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline
  run b512 --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline
done
run dp_b512_graph --dp --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run dp_world1 --dp --steps 100 --warmup 10 --no-cpu-baseline
