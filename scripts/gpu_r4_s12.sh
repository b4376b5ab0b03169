#!/bin/bash
# Round 4: device rounds over base + pending delta run (no compaction on a read) -- the round
# tests, the tier-off write -> round cycle at 10^8, interleaves with the tier off and with the
# no-wait tier policy, and the rbsr line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s12
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests/test_rbsr.py tests/test_rbsr_latency.py tests/test_tier_interleave.py -m gpu -q -rf --timeout 300 --timeout-method thread
run latency 400 bash -c 'reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 0 1 && reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1'
run interleave_off 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 0 c5 2 3
run interleave_nowait 400 env RSOS_HIP_TIER_SYNC=0 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
run rbsr 300 python3 bench.py --config rbsr
echo "== done"
