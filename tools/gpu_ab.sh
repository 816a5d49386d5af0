#!/bin/bash
# Fused-MLP microbench (precisions in $MB_PRECS, default bf16) for the default library
# and each named variant, then (RUN_TESTS=1) the MLP parity tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${MB_PRECS:-bf16}
timeout -k 10 300 python tools/microbench_mlp.py $P > gpurun_out/mb_default.log 2>&1 || { tail -20 gpurun_out/mb_default.log; exit 3; }
echo "== default"; grep -E "^(bf16|fp16|fp32)" gpurun_out/mb_default.log
for v in "$@"; do
  NR_HIP_LIB=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v timeout -k 10 300 python tools/microbench_mlp.py $P > gpurun_out/mb_$v.log 2>&1 || { tail -20 gpurun_out/mb_$v.log; exit 4; }
  echo "== $v"; grep -E "^(bf16|fp16|fp32)" gpurun_out/mb_$v.log
done
if [ "${RUN_TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_parity_mlp.py tests/test_parity_fullsize.py tests/test_determinism.py tests/test_fused_optim.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_ab.log 2>&1
  echo "pytest rc=$?"; tail -3 gpurun_out/pt_ab.log
fi
