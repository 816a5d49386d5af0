#!/bin/bash
# Round 5: GraphedTrainer copies its static inputs in one launch; the graph-replay tests
# and the 512-ray graph step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_coarse_stream.py tests/test_fused_optim.py tests/test_entry_points.py tests/test_rccl.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5o_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r5o_pytest.log; [ $rc = 0 ] || exit 2
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --batch 512 --graph --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/r5o_b512g_$i.json 2> gpurun_out/r5o_b512g_$i.err || { tail -n 20 gpurun_out/r5o_b512g_$i.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/r5o_b512g_$i.json'));print('b512g', d['value'], d['ms_per_step'])"
done
