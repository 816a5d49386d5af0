#!/bin/bash
# Round 5, first box: the GPU suite on this tree, then the fused-vs-split microbench for
# the default library and the ring-depth variants named on the command line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5a_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5a_pytest.log; [ $rc = 0 ] || exit 2
MB_KERNELS=bwd_dx,bwd_dw,bwd_dxdw,bwd_dx,bwd_dw,bwd_dxdw timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/r5a_mb_default.log 2>&1 || { tail -20 gpurun_out/r5a_mb_default.log; exit 3; }
echo "== default"; grep -E "^bf16" gpurun_out/r5a_mb_default.log
for v in "$@"; do
  NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v MB_KERNELS=bwd_dxdw,bwd_dxdw,bwd_dxdw timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/r5a_mb_$v.log 2>&1 || { tail -20 gpurun_out/r5a_mb_$v.log; exit 4; }
  echo "== $v"; grep -E "^bf16" gpurun_out/r5a_mb_$v.log
done
