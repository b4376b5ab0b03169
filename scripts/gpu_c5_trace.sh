#!/bin/bash
# config5 kernel trace (per-kernel timestamps) for a per-batch breakdown of the incremental path
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5t
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5t -o c5 -- \
  python bench.py --config config5 --steps 20 --warmup 3 --cpu-baseline 0 --spinup-ms 0 ${EXTRA:-} \
  > gpurun_out/c5t.log 2>&1 || { echo "trace failed: $?"; tail -20 gpurun_out/c5t.log; exit 1; }
grep -h '"metric"' gpurun_out/c5t.log | cut -c1-300
find gpurun_out/c5t -name "*kernel_trace.csv" | head
