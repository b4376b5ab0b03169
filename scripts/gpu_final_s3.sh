#!/bin/bash
# Round-2 closing session: every -m gpu test, smoke, the default bench line (config4, 100 M), its
# rocprofv3 kernel stats (headline launches only), the config5 line, the one-rank RCCL path of
# every workload and the reconciliation_drive latency harness.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '"metric"\|passed\|failed\|smoke' "$O/$name.log" | cut -c1-300 | tail -3
  [ $rc -eq 0 ] || exit $rc
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python bench.py
run bench_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --cpu-baseline 0 --e2e 0
run config5 300 python bench.py --config config5
run config5_40 300 python bench.py --config config5 --steps 40 --cpu-baseline 0
run rccl1 900 bash scripts/gpu_rccl1.sh
run latency 300 bash -c 'for t in 0 1; do for d in 1 100; do reconcile-rs_amd/examples/rbsr_latency 1000000 $d 500 $t || exit 1; done; done'
echo "== done"
