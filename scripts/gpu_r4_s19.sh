#!/bin/bash
# Round 4, final GPU session (larger rounds emitted into mapped memory): every GPU test, smoke, the default and config5
# lines, the tier interleave (large batches; then small writes after them) and the 1-row write ->
# round cycle at 10^8.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s19
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run pytest_gpu 700 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread
run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
run default 300 python3 bench.py
run c5_20 300 python3 bench.py --config config5
run interleave 300 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run interleave_small 300 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
run latency 200 reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1
run latency_off 200 reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 0 1
run rbsr 300 python3 bench.py --config rbsr
echo "== done"
