#!/bin/bash
# search-table build change: every -m gpu test, then a config5 kernel trace (k_search_table durations)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 bench.py --config config5 --cpu-baseline 0 > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
grep -h '"metric"' $O/prof.log | cut -c1-200
grep k_search_table $O/prof/c5_kernel_stats.csv | cut -c1-200
