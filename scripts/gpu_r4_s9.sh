#!/bin/bash
# Round 4, ninth GPU session: the small path and device rounds with cached device addresses --
# their tests, then the 1-row write -> round cycle at 10^6 and 10^8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s9
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests/test_small_batch.py tests/test_rbsr.py tests/test_rbsr_latency.py tests/test_insert_latency.py tests/test_gpu_parity.py -k "small or rbsr or round or insert or staged or variants or host_tier" -m gpu -q -rf --timeout 300 --timeout-method thread
run latency 400 bash -c 'reconcile-rs_amd/examples/rbsr_latency 1000000 1 300 1 1 && reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1 && reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 0 1'
echo "== done"
