#!/bin/bash
# Pipeline iteration: fused-vs-split bit identity first (any failure ends the session),
# then the per-stage timing records of the diagnostic build, then fused vs split bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pipe.py -m gpu -q -p no:cacheprovider -x \
  --timeout 200 --timeout-method thread > gpurun_out/r04_pipe_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r04_pipe_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -40 gpurun_out/r04_pipe_pytest.log; exit $rc; fi
timeout -k 10 200 python tools/pipe_flaky.py 12807 262144 786432 > gpurun_out/r04_pipeflaky.txt 2>&1
rc=$?
grep "reps" gpurun_out/r04_pipeflaky.txt
if [ $rc -ne 0 ]; then echo "flaky rc=$rc"; tail -20 gpurun_out/r04_pipeflaky.txt; exit $rc; fi
NR_HIP_LIB=robust-nerf_amd/noisy_src/lib/variants/pipeprof timeout -k 10 120 python tools/pipe_prof.py > gpurun_out/r04_pipeprof.txt 2>&1
rc=$?
cat gpurun_out/r04_pipeprof.txt
if [ $rc -ne 0 ]; then echo "prof rc=$rc"; exit $rc; fi
NR_MLP_BACKWARD=fused timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r04_pipe_bench.json 2> gpurun_out/r04_pipe_bench.err
rc=$?
if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -20 gpurun_out/r04_pipe_bench.err; exit $rc; fi
python -c "import json;d=json.load(open('gpurun_out/r04_pipe_bench.json'));print('fused', d['value'], d['ms_per_step'])"
