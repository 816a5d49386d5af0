#!/bin/bash
# Round-4 DP session: the RCCL tests (world-1 group, DP step == plain step, captured
# all-reduce), then bench lines of the 512-ray per-rank DP step over RCCL (eager, graph)
# and the default cfg #2 line.  Any failure ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rccl.py tests/test_fused_optim.py -m gpu -v -p no:cacheprovider \
  --timeout 500 --timeout-method thread > gpurun_out/r04_rccl_pytest.log 2>&1
rc=$?
tail -12 gpurun_out/r04_rccl_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/r04_$n.json 2> gpurun_out/r04_$n.err
  local r=$?
  if [ $r -ne 0 ]; then echo "bench $n rc=$r"; tail -20 gpurun_out/r04_$n.err; exit 5; fi
  python -c "import json;d=json.load(open('gpurun_out/r04_$n.json'));print('$n', d['value'], d['ms_per_step'], d['config']['parallelism'])"
}
run dp_b512 --dp --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline
run dp_b512_graph --dp --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run b512_graph --global-batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run default --steps 50 --warmup 10 --no-cpu-baseline
