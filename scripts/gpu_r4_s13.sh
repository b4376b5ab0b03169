#!/bin/bash
# Round 4: reads over base + pending delta run (rounds, select, key dumps, rank-range aggregates,
# the two-call round steps) with the run's sums taken from block sums -- the tests, the tier-off
# write -> round cycle at 10^8, the tier-off interleave, and a kernel summary of a short one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s13
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest 700 python -u -m pytest tests/test_rbsr.py tests/test_rbsr_latency.py tests/test_tier_interleave.py tests/test_gpu_parity.py -k "rbsr or round or lsm or tier or run_copy or interleave or latency or select or split or resolve" -m gpu -q -rf --timeout 300 --timeout-method thread
run latency 400 reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 0 1
run interleave_off 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 0 c5 2 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- reconcile-rs_amd/examples/tier_interleave 100000000 1000000 4 0 c5 1 3 > $O/prof.log 2>&1 || exit $?
python3 scripts/copy_summary.py $O/prof > $O/interleave_off_kernel_stats.txt 2>&1 || true
rm -rf $O/prof/*/*_kernel_trace.csv 2>/dev/null
RSOS_HIP_TIER_SYNC=0 timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/hip -o hip -- reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3 > $O/nowait_trace.log 2>&1 || exit $?
python3 scripts/long_calls.py $O/hip > $O/nowait_long_calls.txt 2>&1 || true
rm -rf $O/hip
echo "== done"
