#!/bin/bash
# config5 compaction threshold sweep: 64 batches of 1 M into 100 M at divisors 8 / 6 / 5 / 4
# (threshold = base rows / divisor), per-batch wall time through the Python API
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5div
for d in 8 6 5 4; do
  timeout -k 10 300 python scripts/c5_host_probe.py 100000000 $d 64 > gpurun_out/c5div/div$d.log 2>&1 || { echo "div $d failed"; tail -5 gpurun_out/c5div/div$d.log; exit 1; }
  echo "div $d: $(tail -1 gpurun_out/c5div/div$d.log)"
done
