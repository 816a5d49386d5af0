#!/bin/bash
# (Ran against the NR_RBM_WAVES patch of DESIGN.md section 9 item 7, since reverted: the
#  variant libraries it names no longer build from this tree.)
# Same-box A/B of the 512-ray graph-replayed step: size-selected wave count (default
# library) vs forced 8 waves (variant rbm8), alternating, two runs each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/robust-nerf_amd/noisy_src/lib/variants
for i in 1 2; do
  for v in auto rbm8; do
    if [ $v = auto ]; then L=""; else L=$V/$v; fi
    NR_HIP_LIB=$L timeout -k 10 300 python bench.py --global-batch 512 --steps 300 --warmup 20 --no-cpu-baseline --graph > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { tail -20 gpurun_out/ab_$v$i.err; exit 2; }
    python -c "
import json; d=json.load(open('gpurun_out/ab_$v$i.json')); print('$v$i', d['value'], d['ms_per_step'], d['step_ms_p10_p50_p90'])"
  done
done
