#!/bin/bash
# Round-4 closing session for the final tree: the fused-path tests (bit identity), smoke,
# then tools/gpu_profile.sh (default bench + rocprofv3 kernel trace + HBM PMC passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pipe.py tests/test_rccl.py -m gpu -q -p no:cacheprovider -x \
  --timeout 300 --timeout-method thread > gpurun_out/r04_final_pipe_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r04_final_pipe_pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
bash tools/gpu_profile.sh || exit 2
