#!/bin/bash
# store iteration: the store / sort / incremental GPU tests, then a config5 kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_emap.py tests/test_fmap.py -k "${K:-store or incremental or emap or fmap or host_tier}" \
  > gpurun_out/store_iter.log 2>&1 || { echo "store tests failed: $?"; tail -30 gpurun_out/store_iter.log; exit 1; }
tail -2 gpurun_out/store_iter.log
bash scripts/gpu_c5_trace.sh
