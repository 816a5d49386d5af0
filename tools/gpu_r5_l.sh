#!/bin/bash
# Round 5: where the fp32 training forward's time goes -- timing-only variants (wrong
# results): no saved-activation stores in the stream, no weight-stream DMA, no chunk
# barriers; fine M, alternating with the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/robust-nerf_amd/noisy_src/lib/variants
for i in 1 2; do
  for v in default f_nosink f_nodma f_nobar; do
    lib=""; [ $v = default ] || lib=$V/$v
    NR_HIP_LIB=$lib MB_REPS=3 MB_KERNELS=fwd_train,fwd_train,bwd_dx timeout -k 10 300 python tools/microbench_mlp.py fp32 > gpurun_out/r5l_${v}_$i.log 2>&1 || { tail -n 20 gpurun_out/r5l_${v}_$i.log; exit 3; }
    echo "== $v $i"; grep -E "^fp32" gpurun_out/r5l_${v}_$i.log
  done
done
