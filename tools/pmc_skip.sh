#!/bin/bash
# HBM bytes per launch of the fine dX / dW kernels, dense vs skipping (MB_ACTIVE=0.37,
# ray-shaped activity): two PMC passes per mode (FETCH_SIZE, WRITE_SIZE; separate runs),
# over tools/microbench_mlp.py.  Output: gpurun_out/pmc_skip_<mode>_<counter>/.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp MB_KERNELS=bwd_dx,bwd_dw MB_REPS=3
for mode in dense skip; do
  if [ $mode = skip ]; then export MB_ACTIVE=0.37 MB_PATTERN=rays; else unset MB_ACTIVE MB_PATTERN; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_skip_${mode}_$c -o run --output-format csv -- \
      python tools/microbench_mlp.py bf16 > gpurun_out/pmc_skip_${mode}_$c.log 2>&1 || { echo "pass $mode $c failed"; tail -5 gpurun_out/pmc_skip_${mode}_$c.log; exit 1; }
  done
done
echo done
