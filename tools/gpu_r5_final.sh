#!/bin/bash
# Round-5 closing session on the final tree: the full GPU suite, then tools/gpu_profile.sh
# (smoke, default bench, rocprofv3 kernel trace, HBM PMC passes), then the world-1 RCCL
# data-parallel line (topology fields) and its kernel trace (all-reduce overlap).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05_final_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/r05_final_pytest.log; [ $rc = 0 ] || exit 2
bash tools/gpu_profile.sh || exit 3
timeout -k 10 300 python bench.py --dp --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/r05_bench_dp_world1.json 2> gpurun_out/r05_bench_dp_world1.err || { tail -n 20 gpurun_out/r05_bench_dp_world1.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/r05_bench_dp_world1.json'));print('dp', d['value'], d['ms_per_step'], d.get('topology'))"
rm -rf gpurun_out/prof_dp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_dp -o run --output-format csv -- python bench.py --dp --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_dp.log 2>&1 || { tail -n 20 gpurun_out/prof_dp.log; exit 5; }
python tools/overlap_trace.py gpurun_out/prof_dp gpurun_out/r05_dp_overlap.txt | tail -n 3
# multi-rank rehearsal: 4 ranks sharing the one GPU over gloo (RCCL refuses two ranks on
# one device); the same barriers, max-over-ranks timing, aggregate value and topology
NR_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05_bench_gloo4.json 2> gpurun_out/r05_bench_gloo4.err || { tail -n 20 gpurun_out/r05_bench_gloo4.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/r05_bench_gloo4.json'));print('gloo4', d['value'], d['n_gpus'], d['config']['parallelism'], [ (r['rank'], r['device'], r['step_ms_median']) for r in d['topology']['ranks']])"
