#!/bin/bash
# store iteration: every -m gpu test, the default config5 line, 64 batches through the probe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread \
  > gpurun_out/sc/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" gpurun_out/sc/tests.log | head -20; tail -5 gpurun_out/sc/tests.log; exit 1; }
tail -1 gpurun_out/sc/tests.log
timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 > gpurun_out/sc/c5_20.log 2>&1 || { echo "c5 bench failed"; exit 1; }
grep -h '"metric"' gpurun_out/sc/c5_20.log | cut -c1-200
timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --steps 40 > gpurun_out/sc/c5_40.log 2>&1 || { echo "c5 bench 40 failed"; exit 1; }
grep -h '"metric"' gpurun_out/sc/c5_40.log | cut -c1-200
timeout -k 10 300 python scripts/c5_host_probe.py 100000000 8 64 > gpurun_out/sc/c5_probe64.log 2>&1 || { echo "probe failed"; exit 1; }
tail -1 gpurun_out/sc/c5_probe64.log
