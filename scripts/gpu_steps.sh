#!/bin/bash
# Ad-hoc GPU session: each argument pair is  name 'command'; every step runs under its own
# timeout, logs to gpurun_out/<name>.log, and the session stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${STEP_TIMEOUT:-300}
while [ $# -ge 2 ]; do
  name=$1; cmd=$2; shift 2
  echo "== $name: $cmd"
  timeout -k 10 "$T" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping at $name ($rc)"; exit $rc; }
done
echo "== done"
