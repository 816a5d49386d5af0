#!/bin/bash
# GPU session: smoke, bench (default), rocprofv3 kernel stats of a short bench,
# then the two HBM PMC passes (FETCH_SIZE / WRITE_SIZE: separate passes, TCC slots).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
# the kernel trace runs the driver's bench command (20 timed steps after 5 warm-up steps):
# tools/prof_summary.py ... 20 averages each fused-MLP kernel over its timed launches
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -30 gpurun_out/pmc_write.log; exit 1; }
find gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.csv" | head -20
