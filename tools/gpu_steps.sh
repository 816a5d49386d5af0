#!/bin/bash
# GPU-box driver: run named steps in order, each under its own time limit, its output in
# gpurun_out/<name>.log.  A step that fails normally (exit 1: a failing test) lets the
# next one run; anything else (a fault, an abort, a time limit) stops the call there.
#
#   tools/gpu_steps.sh 'name|seconds|command' ['name|seconds|command' ...]
#
# e.g. tools/gpu_steps.sh 'tests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
#                         'bench|300|python -u bench.py --steps 50'
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then
    status=$rc
    if [ $rc -ne 1 ]; then
      echo "== stopping after $name (rc=$rc)"
      exit $rc
    fi
  fi
done
exit $status
