#!/bin/bash
# Round-2 GPU session: every -m gpu test, smoke, the default bench line (config4: 100 M records,
# north_star shape), the one-rank RCCL path of every workload, the reconciliation_drive latency
# harness and the staged-insert probe.  Stops at the first fatal step (timeout / signal).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "fatal step $name ($rc)"; exit $rc; fi
  return 0
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
run rccl1 900 bash scripts/gpu_rccl1.sh
run latency 300 bash -c 'for t in 0 1; do for d in 1 100; do reconcile-rs_amd/examples/rbsr_latency 1000000 $d 500 $t || exit 1; done; done'
run fmap_probe 300 python scripts/fmap_probe.py
echo "== done"
