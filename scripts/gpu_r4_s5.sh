#!/bin/bash
# Round 4, fifth GPU session: every GPU test, smoke, the default and config5 lines (config5's
# traffic now from r04_pmc_config5.json), the tier interleave with the run copy's select index,
# and the 1-row write -> round cycle at 10^8.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R4_OUT:-r4s5}
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
run interleave_default 300 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run latency 200 reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1
echo "== done"
