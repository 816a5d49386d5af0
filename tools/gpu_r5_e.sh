#!/bin/bash
# Round 5: per-stage in-kernel timing of the 8-wave pipeline with timing-only variants:
# no dz ring / staging traffic, no hand-off waits, neither.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pipeprof pp_neither pp_nowait pp_all; do
  NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v timeout -k 10 200 python tools/pipe_prof.py > gpurun_out/r5e_$v.log 2>&1 || { tail -20 gpurun_out/r5e_$v.log; exit 4; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r5e_$v.log
done
