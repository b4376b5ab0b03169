#!/bin/bash
# encoded-lift iteration: its parity tests, the timing probe, then a kernel trace of 64 config5
# batches into 100 M (compactions at a growing base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/enc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_emap.py -q -x --timeout 120 --timeout-method thread \
  -k "encoded or fixed or emap or golden" > gpurun_out/enc/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/enc/tests.log; exit 1; }
tail -1 gpurun_out/enc/tests.log
timeout -k 10 300 python3 scripts/encoded_probe.py > gpurun_out/enc/probe.log 2>&1 || { echo "probe failed"; exit 1; }
cat gpurun_out/enc/probe.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/enc/c5 -o c5 -- python3 scripts/c5_host_probe.py 100000000 8 64 \
  > gpurun_out/enc/c5.log 2>&1 || { echo "c5 trace failed"; exit 1; }
tail -1 gpurun_out/enc/c5.log
