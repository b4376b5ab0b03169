#!/bin/bash
# Round 3: the whole GPU suite, then smoke()
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3_full
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -n 5 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; exit $rc
