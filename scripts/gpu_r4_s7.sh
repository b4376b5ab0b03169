#!/bin/bash
# Round 4, seventh GPU session: small writes after large batches (folds over the run copy) --
# the tests, and the interleave at 10^8 with 3 single-row writes after each 1 M-row batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s7
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest_tier 500 python -u -m pytest tests/test_tier_interleave.py tests/test_gpu_parity.py -k "interleave or small_writes or run_copy or host_tier" -m gpu -v --timeout 300 --timeout-method thread
run interleave_small 500 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
run latency 200 reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1
run interleave_small_tier0 500 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 0 c5 2 3
echo "== done"
