#!/bin/bash
# Round 4: the tier refresh's scans on the copy stream -- tier and round tests, then the default,
# no-wait and tier-off interleaves (3 small cycles after each 1 M-row batch) at 10^8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s15
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest 700 python -u -m pytest tests/test_tier_interleave.py tests/test_rbsr.py tests/test_gpu_parity.py -k "tier or run_copy or host_tier or interleave or rbsr or round or lsm or policy" -m gpu -q -rf --timeout 300 --timeout-method thread
run interleave_sync 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
run interleave_nowait 400 env RSOS_HIP_TIER_SYNC=0 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
run interleave_off 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 0 c5 2 3
echo "== done"
