#!/bin/bash
# Round 4, first GPU session: the torch 10^8-row repro, the small-batch path's
# tests and the store tests, kernel + copy traces of the 1-row write -> round cycle with the small
# path off (the round-3 baseline) and on, the write -> round cycle at 10^8 and the insert harness.
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s1
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || [ "${OKRC:-0}" = "$rc" ] || exit $rc
}
run pytest_small 240 python -u -m pytest tests/test_small_batch.py -m gpu -x -v --timeout 300 --timeout-method thread
run pytest_all 650 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread
for v in off on; do
  if [ $v = off ]; then export RSOS_HIP_SMALL_MAX=0; else unset RSOS_HIP_SMALL_MAX; fi
  run write_trace_$v 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/wt_$v -o wt -- reconcile-rs_amd/examples/rbsr_latency 1000000 1 60 1 1
  python3 scripts/write_timeline.py $O/wt_$v k_merge_run > $O/write_timeline_$v.txt 2>&1
  tail -30 $O/write_timeline_$v.txt
  rm -rf $O/wt_$v
  run latency_$v 600 bash -c 'reconcile-rs_amd/examples/rbsr_latency 1000000 1 300 1 1 && reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 1 1'
done
OKRC=1 run torch_repro 240 python -u scripts/torch_large_ops_repro.py 100000000  # 1: a check disagreed
echo "== done"
