#!/bin/bash
# Round-end GPU session for profiles/: the -m gpu suite, smoke, the default bench with
# its rocprofv3 kernel trace and HBM PMC passes (tools/gpu_profile.sh), then one bench
# line per BASELINE config.  Any failure ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  NR_PARITY_OUT=$PWD/gpurun_out/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
bash tools/gpu_profile.sh || exit 2
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/b_$n.json 2> gpurun_out/b_$n.err
  local r=$?
  if [ $r -ne 0 ]; then echo "bench $n rc=$r"; tail -20 gpurun_out/b_$n.err; exit 5; fi
  python -c "import json;d=json.load(open('gpurun_out/b_$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
run b512 --batch 512 --steps 100 --warmup 10 --no-cpu-baseline
run b512_graph --batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run pose_opt --pose-opt --steps 20 --warmup 5
run cfg5_fp16 --precision fp16 --num-samples 128 --num-samples-fine 256 --steps 20 --warmup 5 --no-cpu-baseline
run fp32 --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline
run eval --eval
