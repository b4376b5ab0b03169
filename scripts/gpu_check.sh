#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.  Stops at the first
# step that faults / aborts / times out (exit >= 124 or signal); test failures (exit 1)
# are recorded and the session continues so the bench evidence is still collected.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "fatal step $name ($rc): stopping"; exit $rc; fi
  return 0
}
run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps "$STEPS" --warmup 5 --e2e 1
run rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps "$STEPS" --warmup 5 --cpu-baseline 0 --check 0 --e2e 0
echo "== done"
