#!/bin/bash
# Round 4: the tree as committed at the end of the round -- every GPU test, smoke, the default line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s23
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run pytest_gpu 700 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread
run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
run default 300 python3 bench.py
echo "== done"
