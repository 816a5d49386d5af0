#!/bin/bash
# Round-4 profile session: smoke + default bench + rocprofv3 kernel trace + HBM PMC
# passes (tools/gpu_profile.sh), the per-config bench lines, then the opt-in fused
# layer-pipelined backward (NR_MLP_BACKWARD=fused) as a same-box A/B with its own trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_profile.sh || exit 2
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/b_$n.json 2> gpurun_out/b_$n.err
  local r=$?
  if [ $r -ne 0 ]; then echo "bench $n rc=$r"; tail -20 gpurun_out/b_$n.err; exit 5; fi
  python -c "import json;d=json.load(open('gpurun_out/b_$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
run split_ab --steps 50 --warmup 10 --no-cpu-baseline
NR_MLP_BACKWARD=fused run fused_ab --steps 50 --warmup 10 --no-cpu-baseline
rm -rf gpurun_out/fused && mkdir -p gpurun_out/fused
NR_MLP_BACKWARD=fused timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/fused/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fused/prof.log 2>&1 || { echo "fused rocprof failed"; tail -20 gpurun_out/fused/prof.log; exit 6; }
run b512_graph --batch 512 --steps 100 --warmup 10 --no-cpu-baseline --graph
run pose_opt --pose-opt --steps 20 --warmup 5
run cfg5_fp16 --precision fp16 --num-samples 128 --num-samples-fine 256 --steps 20 --warmup 5 --no-cpu-baseline
run eval --eval
