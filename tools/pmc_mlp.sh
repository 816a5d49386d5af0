#!/bin/bash
# PMC passes over the fused-MLP microbench ($MB_PREC, default bf16; M=786432): one rocprofv3 run per
# counter set (gfx950 slot limits: <=8 SQ, <=4 TCC per pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp MB_REPS=3
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for set in "$@"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc$i -o run --output-format csv -- python tools/microbench_mlp.py ${MB_PREC:-bf16} > gpurun_out/pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc$i.log; exit 1; }
done
find gpurun_out -name "*counter_collection.csv" | head
