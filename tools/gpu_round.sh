#!/bin/bash
# One GPU session: the -m gpu suite (collect every failure), then tools/gpu_profile.sh
# (smoke, bench, rocprofv3 kernel stats, FETCH/WRITE PMC passes) with the given bench args.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/gpu_profile.sh "$@" || exit $?
exit $rc
