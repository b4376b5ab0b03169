#!/bin/bash
# the whole GPU suite, then a config5 kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests \
  > gpurun_out/full_iter.log 2>&1 || { echo "gpu tests failed: $?"; grep -E "FAILED|Error|error" gpurun_out/full_iter.log | head -30; tail -5 gpurun_out/full_iter.log; exit 1; }
tail -2 gpurun_out/full_iter.log
bash scripts/gpu_c5_trace.sh
