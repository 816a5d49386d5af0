#!/bin/bash
# Round 5: per-job dW workgroup counts for fp32 -- the GPU suite, then the fp32 dW A/B
# (this library vs the uniform grid of the previous commit, alternating) and the fp32
# cfg #2 step.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r5g_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5g_pytest.log; [ $rc = 0 ] || exit 2
for i in 1 2; do
  for v in default head_uniform_dw; do
    lib=""; [ $v = default ] || lib=$PWD/robust-nerf_amd/noisy_src/lib/variants/$v
    NR_HIP_LIB=$lib MB_REPS=5 MB_KERNELS=bwd_dw,bwd_dw timeout -k 10 300 python tools/microbench_mlp.py fp32 > gpurun_out/r5g_mb_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5g_mb_${v}_$i.log; exit 3; }
    echo "== $v $i"; grep -E "^fp32" gpurun_out/r5g_mb_${v}_$i.log
  done
done
timeout -k 10 400 python bench.py --precision fp32 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r5g_bench_fp32.json 2> gpurun_out/r5g_bench_fp32.err || { tail -20 gpurun_out/r5g_bench_fp32.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/r5g_bench_fp32.json'));print('fp32', d['value'], d['ms_per_step'], d['kernel_ms'])"
