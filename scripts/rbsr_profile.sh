#!/bin/bash
# Kernel-trace profile of whole reconciliations (scripts/rbsr_probe.py at d = 1e5) -- the source
# of profiles/r01_rbsr_d100k_kernel_stats.txt.  Probe timings first, then the traced run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/rbsr_probe.py --cpu-n 0 > gpurun_out/rbsr_probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rbsr_prof -o rbsr -- python3 -u scripts/rbsr_probe.py --cpu-n 0 --d 100000 > gpurun_out/rbsr_prof.log 2>&1
