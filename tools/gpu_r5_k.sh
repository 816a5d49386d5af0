#!/bin/bash
# Round 5: coarse_stream="auto" (bench default, train.py): GPU tests of the paths it
# touches, then the 512-ray graph step under auto (engages) and 4096 eager (does not).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_coarse_stream.py tests/test_rccl.py tests/test_entry_points.py tests/test_fused_optim.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5k_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r5k_pytest.log; [ $rc = 0 ] || exit 2
for tag in "b512g:--batch 512 --graph --steps 200 --warmup 20" "b512g_off:--batch 512 --graph --steps 200 --warmup 20 --coarse-stream off" "b4096:--steps 50 --warmup 10"; do
  n=${tag%%:*}; a=${tag#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > gpurun_out/r5k_$n.json 2> gpurun_out/r5k_$n.err || { tail -n 20 gpurun_out/r5k_$n.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/r5k_$n.json'));print('$n', d['value'], d['ms_per_step'], d['config'].get('coarse_stream'))"
done
