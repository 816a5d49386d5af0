#!/bin/bash
# Round 5: the coarse chain on a second stream (cfg #4's 512-ray per-rank step) -- tests,
# then a same-box A/B of the graph-replayed step (alternating), and the 4096-ray default.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_coarse_stream.py tests/test_fused_optim.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5f_pytest.log; [ $rc = 0 ] || exit 2
for i in 1 2; do
  for cs in "" "--coarse-stream"; do
    tag=b512g${cs:+_cs}_$i
    timeout -k 10 300 python bench.py --batch 512 --graph $cs --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/r5f_$tag.json 2> gpurun_out/r5f_$tag.err || { tail -20 gpurun_out/r5f_$tag.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/r5f_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])"
  done
done
for cs in "" "--coarse-stream"; do
  tag=b4096${cs:+_cs}
  timeout -k 10 300 python bench.py $cs --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r5f_$tag.json 2> gpurun_out/r5f_$tag.err || { tail -20 gpurun_out/r5f_$tag.err; exit 4; }
  python -c "import json;d=json.load(open('gpurun_out/r5f_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
done
