#!/bin/bash
# Round 4, session 1b: the host-tier tests after the no-wait refresh policy, the 1-row write -> round
# cycle with the small path off (round 3's path) and on (kernel + copy traces, then latencies at 10^6
# and 10^8), the tier under 1 M-row batches at 10^8, the staged-insert harness, the torch 10^8 repro.
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s1b
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || [ "${OKRC:-0}" = "$rc" ] || exit $rc
}
run pytest_tier 400 python -u -m pytest tests/test_gpu_parity.py -k "host_tier or write_round or staged" tests/test_tier_interleave.py tests/test_insert_latency.py tests/test_rbsr_latency.py -m gpu -v --timeout 300 --timeout-method thread
for v in off on; do
  if [ $v = off ]; then export RSOS_HIP_SMALL_MAX=0; else unset RSOS_HIP_SMALL_MAX; fi
  run write_trace_$v 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/wt_$v -o wt -- reconcile-rs_amd/examples/rbsr_latency 1000000 1 60 1 1
  python3 scripts/write_timeline.py $O/wt_$v k_merge_run > $O/write_timeline_$v.txt 2>&1
  tail -30 $O/write_timeline_$v.txt
  rm -rf $O/wt_$v
  run latency_$v 600 bash -c 'reconcile-rs_amd/examples/rbsr_latency 1000000 1 300 1 1 && reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 1 1'
done
run inserts 300 bash -c 'reconcile-rs_amd/examples/insert_latency 100000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 0'
run interleave_c5_1m_tier1 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 1 c5 2
run interleave_c5_1m_tier0 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 20 0 c5 2
OKRC=1 run torch_repro 240 python -u scripts/torch_large_ops_repro.py 100000000  # 1: a check disagreed
echo "== done"
