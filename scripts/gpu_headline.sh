#!/bin/bash
# smoke + the default bench line (config4 100 M, N=1) + its rocprofv3 kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/hl
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/hl/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/hl/smoke.log; exit 1; }
tail -1 gpurun_out/hl/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/hl/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/hl/bench.log; exit 1; }
grep -h '"metric"' gpurun_out/hl/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hl/prof -o run -- python3 bench.py --cpu-baseline 0 > gpurun_out/hl/prof.log 2>&1 || { echo "prof failed"; exit 1; }
head -3 gpurun_out/hl/prof/run_kernel_stats.csv
