#!/bin/bash
# Round-3 GPU session: the -m gpu suite (every failure collected, parity records to
# gpurun_out/parity.jsonl), then bench lines: cfg #2 default, the eval path, the fp32
# parity mode and cfg #4's 512-ray per-rank workload.  Each GPU step has its own limit;
# a fault/abort/timeout ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/parity.jsonl
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  NR_PARITY_OUT=$PWD/gpurun_out/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/b_$n.json 2> gpurun_out/b_$n.err
  local r=$?
  if [ $r -ne 0 ]; then echo "bench $n rc=$r"; tail -20 gpurun_out/b_$n.err; exit 5; fi
  echo "== $n"; cat gpurun_out/b_$n.json
}
run cfg2 --steps 20 --warmup 5
run eval --eval
run fp32 --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline
run b512 --batch 512 --steps 100 --warmup 10 --no-cpu-baseline
exit ${rc:-0}
