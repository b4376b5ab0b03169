#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/snap_prof
timeout -k 10 300 python3 bench.py --config snapshot > gpurun_out/snap_prof/bench.log 2>&1; rc=$?
grep -h '"metric"' gpurun_out/snap_prof/bench.log | cut -c1-3000; tail -3 gpurun_out/snap_prof/bench.log | cut -c1-300; exit $rc
