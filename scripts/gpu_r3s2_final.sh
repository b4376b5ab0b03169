#!/bin/bash
# Round 3, second session, closing measurements: every -m gpu test, smoke, the default bench line
# (config4, 100 M) and its kernel stats, config2, snapshot, encoded, config5 lines (20 / 40 / 64
# batches) with a kernel trace, the 100 M-resident config5 test, and the latency harnesses.
# Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3s2_final
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '"metric"\|passed\|failed\|smoke' "$O/$name.log" | cut -c1-300 | tail -3
  [ $rc -eq 0 ] || exit $rc
}
[ "${SKIP_TESTS:-0}" = 0 ] && run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python bench.py
run bench_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --cpu-baseline 0 --e2e 0
find $O/stats -name "*kernel_stats.csv" -exec cp {} $O/config4_kernel_stats.csv \; ; rm -rf $O/stats
run config2 300 python bench.py --config config2
run snapshot 300 python bench.py --config snapshot
run encoded 300 python bench.py --config encoded
run config5 300 python bench.py --config config5
run config5_40 300 python bench.py --config config5 --steps 40 --cpu-baseline 0
run config5_64 300 python bench.py --config config5 --steps 64 --cpu-baseline 0
run config5_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- python3 bench.py --config config5 --steps 40 --warmup 3 --cpu-baseline 0 --spinup-ms 0
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/c5_timeline.py "$f" 10 20 30 > $O/config5_timeline.txt 2>&1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/config5_kernel_stats.csv \; ; rm -rf $O/trace
run latency 600 bash -c 'for w in 0 1 1000; do reconcile-rs_amd/examples/rbsr_latency 1000000 1 300 1 $w || exit 1; done; for w in 1 1000; do reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 1 $w || exit 1; done'
run inserts 300 bash -c 'reconcile-rs_amd/examples/insert_latency 100000 1000000 1 && reconcile-rs_amd/examples/insert_latency 10000000 1000000 1'
echo "== done"
