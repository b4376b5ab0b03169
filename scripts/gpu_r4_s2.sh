#!/bin/bash
# Round 4, second GPU session: the small path with its role-split launch and polled completion word,
# the tier's re-pin fix; tests, the 1-row write -> round cycle at 10^6 / 10^8, the insert harness,
# and the tier under 1 M-row batches at 10^8 with a kernel + copy trace.  Stops at the first failing step.
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
run pytest_small 500 python -u -m pytest tests/test_small_batch.py tests/test_gpu_parity.py -k "small or variants or host_tier or write_round or staged or keys_checked" tests/test_insert_latency.py tests/test_tier_interleave.py tests/test_rbsr_latency.py -m gpu -v --timeout 300 --timeout-method thread
run write_trace_on 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/wt_on -o wt -- reconcile-rs_amd/examples/rbsr_latency 1000000 1 60 1 1
python3 scripts/write_timeline.py $O/wt_on k_merge_run > $O/write_timeline_on.txt 2>&1; rm -rf $O/wt_on
run latency_on 600 bash -c 'reconcile-rs_amd/examples/rbsr_latency 1000000 1 300 1 1 && reconcile-rs_amd/examples/rbsr_latency 100000000 1 200 1 1'
run inserts 300 bash -c 'reconcile-rs_amd/examples/insert_latency 100000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 0'
run interleave_trace 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/it -o it -- reconcile-rs_amd/examples/tier_interleave 100000000 1000000 8 1 c5 1
python3 scripts/copy_summary.py $O/it > $O/interleave_copies.txt 2>&1; rm -rf $O/it
run interleave_c5_1m_tier1 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run interleave_c5_1m_tier1_sync 400 env RSOS_HIP_TIER_SYNC=1 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
echo "== done"
