#!/bin/bash
# (Ran against the NR_RBM_WAVES patch of DESIGN.md section 9 item 7, since reverted: the
#  variant libraries it names no longer build from this tree.)
# Row-block-major kernels at 4 vs 8 waves per workgroup: microbench over launch sizes
# (forced-4 / forced-8 variant libraries), the MLP parity tests on the forced-4 build,
# then the default (size-selected) library's tests and 512-ray / cfg #2 bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/robust-nerf_amd/noisy_src/lib/variants
for v in rbm8 rbm4; do
  NR_HIP_LIB=$V/$v MB_M=32768,98304,262144,786432 MB_REPS=30 timeout -k 10 300 python tools/microbench_mlp.py bf16 > gpurun_out/mbw_$v.log 2>&1 || { tail -20 gpurun_out/mbw_$v.log; exit 3; }
  echo "== $v"; grep -E "fwd_train|bwd_dx" gpurun_out/mbw_$v.log
done
NR_HIP_LIB=$V/rbm4 timeout -k 10 600 python -u -m pytest tests/test_parity_mlp.py tests/test_parity_fullsize.py tests/test_determinism.py -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_rbm4.log 2>&1
rc=$?; echo "rbm4 pytest rc=$rc"; tail -2 gpurun_out/pt_rbm4.log; [ $rc -eq 0 ] || exit 4
timeout -k 10 300 python bench.py --global-batch 512 --graph --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b512w.json 2> gpurun_out/b512w.err || { tail -20 gpurun_out/b512w.err; exit 5; }
NR_HIP_LIB=$V/rbm8 timeout -k 10 300 python bench.py --global-batch 512 --graph --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b512w8.json 2> gpurun_out/b512w8.err || { tail -20 gpurun_out/b512w8.err; exit 6; }
python -c "
import json
for f in ['b512w','b512w8']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['kernel_ms'])"
