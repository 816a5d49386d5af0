#!/bin/bash
# Round 5: coarse backward started right after the coarse forward on the coarse stream
# (beside the fine sampling / forward / backward): bit-identity tests, then the 512-ray
# graph step and the 4096-ray step with and without --coarse-stream, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_coarse_stream.py tests/test_rccl.py tests/test_pipe.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5i_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r5i_pytest.log; [ $rc = 0 ] || exit 2
for i in 1 2; do
  for cs in "" "--coarse-stream"; do
    tag=b512g${cs:+_cs}_$i
    timeout -k 10 300 python bench.py --batch 512 --graph --steps 200 --warmup 20 --no-cpu-baseline $cs > gpurun_out/r5i_$tag.json 2> gpurun_out/r5i_$tag.err || { tail -n 20 gpurun_out/r5i_$tag.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/r5i_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
  done
done
for i in 1 2; do
  for cs in "" "--coarse-stream"; do
    tag=b4096${cs:+_cs}_$i
    timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline $cs > gpurun_out/r5i_$tag.json 2> gpurun_out/r5i_$tag.err || { tail -n 20 gpurun_out/r5i_$tag.err; exit 4; }
    python -c "import json;d=json.load(open('gpurun_out/r5i_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"
  done
done
