#!/bin/bash
# HEAD check: every -m gpu test, smoke, the default line and the config5 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/head
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log | cut -c1-200
for k in 20 40; do
  timeout -k 10 300 python bench.py --config config5 --steps $k $( [ $k = 40 ] && echo --cpu-baseline 0 ) > $O/config5_$k.log 2>&1 || { echo "config5 $k failed"; exit 1; }
  grep -h '"metric"' $O/config5_$k.log | cut -c1-200
done
