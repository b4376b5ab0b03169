#!/bin/bash
# Round 4, fourth GPU session: the host tier's run copy (a large batch copies the device's delta run
# instead of the whole base) -- its tests, the interleave harness at 10^8 under the default policy
# (writes keep the tier fresh, run copies) and the no-wait one, a kernel + copy trace of the
# interleave, and the 1-row write -> round cycle.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s4
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest_tier 600 python -u -m pytest tests/test_gpu_parity.py -k "host_tier or run_copy or variants or write_round or staged or keys_checked or bunched" tests/test_small_batch.py tests/test_tier_interleave.py tests/test_insert_latency.py tests/test_rbsr_latency.py -m gpu -v --timeout 300 --timeout-method thread
run interleave_default 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run interleave_nowait 400 env RSOS_HIP_TIER_SYNC=0 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run interleave_tier0 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 0 c5 2
run interleave_trace 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/it -o it -- reconcile-rs_amd/examples/tier_interleave 100000000 1000000 8 1 c5 1
python3 scripts/copy_summary.py $O/it > $O/interleave_copies.txt 2>&1; rm -rf $O/it
run latency 300 reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1
run inserts 300 bash -c 'reconcile-rs_amd/examples/insert_latency 100000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 1'
echo "== done"
