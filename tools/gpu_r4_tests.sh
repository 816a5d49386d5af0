#!/bin/bash
# Round-4 GPU test session: the whole -m gpu suite, then smoke.  Any failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
NR_PARITY_OUT=$PWD/gpurun_out/parity.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r04_pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; grep -E "FAILED|Error" gpurun_out/r04_pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
rc=$?
tail -2 gpurun_out/r04_smoke.log
exit $rc
