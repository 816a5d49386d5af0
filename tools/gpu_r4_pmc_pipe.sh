#!/bin/bash
# Issue / clock counters of the fused layer-pipelined backward vs the split pair (one
# rocprofv3 --pmc pass each: 5 SQ + 1 GRBM counters), on short bench runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for mode in split fused; do
  rm -rf gpurun_out/pmc_$mode
  NR_MLP_BACKWARD=$mode timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_$mode -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$mode.log 2>&1 || { echo "pmc $mode failed"; tail -20 gpurun_out/pmc_$mode.log; exit 1; }
done
echo pmc-ok
