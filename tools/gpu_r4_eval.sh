#!/bin/bash
# Inference launch size: the bit-identity test, then the eval bench at the reference's
# 4096-ray launches (NR_EVAL_CHUNK=0) and at the default larger launches.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_render.py -m gpu -q -p no:cacheprovider -x --timeout 200 \
  --timeout-method thread > gpurun_out/r04_eval_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r04_eval_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; tail -30 gpurun_out/r04_eval_pytest.log; exit $rc; fi
for c in 0 32768 65536; do
  NR_EVAL_CHUNK=$c timeout -k 10 300 python bench.py --eval > gpurun_out/r04_eval_$c.json 2> gpurun_out/r04_eval_$c.err || { echo "eval $c failed"; tail -20 gpurun_out/r04_eval_$c.err; exit 5; }
  python -c "import json;d=json.load(open('gpurun_out/r04_eval_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
