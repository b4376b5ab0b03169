#!/bin/bash
# Round 4, second GPU session: the host tier under large write batches at 10^8 (VERDICT r03 item 5:
# examples/tier_interleave.c, config5's shape, both replicas written then reconciled, drive p99),
# and the staged-insert harness (item 2).  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s2
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
run pytest_interleave 400 python -u -m pytest tests/test_tier_interleave.py -m gpu -x -v --timeout 300 --timeout-method thread
run inserts 300 bash -c 'reconcile-rs_amd/examples/insert_latency 100000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 0'
run interleave_c5_1m_tier1 600 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run interleave_c5_50k_tier1 600 reconcile-rs_amd/examples/tier_interleave 100000000 50000 30 1 c5 2
run interleave_c5_1m_tier0 600 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 0 c5 2
echo "== done"
