#!/bin/bash
# fp32 parity-mode dW: parity tests first (any failure ends the session), then the
# cfg #2 fp32 bench line and its rocprof kernel summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_mlp.py tests/test_parity_fullsize.py tests/test_fused_optim.py -m gpu -k "fp32 or plan or model" -q \
  -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/r04_fp32_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r04_fp32_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -40 gpurun_out/r04_fp32_pytest.log; exit $rc; fi
timeout -k 10 400 python bench.py --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04_fp32_bench.json 2> gpurun_out/r04_fp32_bench.err
rc=$?
if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -20 gpurun_out/r04_fp32_bench.err; exit $rc; fi
python -c "import json;d=json.load(open('gpurun_out/r04_fp32_bench.json'));print('fp32', d['value'], d['ms_per_step'], {k:v for k,v in d['kernel_ms'].items() if 'dw' in k})"
