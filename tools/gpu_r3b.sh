#!/bin/bash
# Round-3 session: the -m gpu suite, then tools/gpu_profile.sh (smoke, bench, rocprof
# kernel trace, FETCH_SIZE / WRITE_SIZE passes).  A failure ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  NR_PARITY_OUT=$PWD/gpurun_out/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
bash tools/gpu_profile.sh "$@"
