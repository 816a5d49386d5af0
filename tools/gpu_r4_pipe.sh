#!/bin/bash
# Round-4 pipeline session: the fused-vs-split backward tests first (any failure ends
# the session), then the full-size step parity and a short bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pipe.py -m gpu -v -p no:cacheprovider -x \
  --timeout 200 --timeout-method thread > gpurun_out/r04_pipe_pytest.log 2>&1
rc=$?
tail -25 gpurun_out/r04_pipe_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
NR_MLP_BACKWARD=fused timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r04_pipe_bench.json 2> gpurun_out/r04_pipe_bench.err
rc=$?
if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -20 gpurun_out/r04_pipe_bench.err; exit $rc; fi
python -c "import json;d=json.load(open('gpurun_out/r04_pipe_bench.json'));print(d['value'], d['ms_per_step'], d['kernel_ms'])"
NR_MLP_BACKWARD=split timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r04_split_bench.json 2> gpurun_out/r04_split_bench.err
python -c "import json;d=json.load(open('gpurun_out/r04_split_bench.json'));print('split', d['value'], d['ms_per_step'], d['kernel_ms'])"
