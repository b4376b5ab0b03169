#!/bin/bash
# Round 3: the fused snapshot reload (snap_lift.hpp) -- snapshot tests, the reload bench line and
# a kernel trace of the reload
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3_snap
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread -m gpu \
  tests/test_snapshot.py > $O/tests.log 2>&1
rc=$?; tail -n 5 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config snapshot --cpu-baseline 0 > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep -h '"metric"' $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o snap -- \
  python bench.py --config snapshot --steps 10 --warmup 2 --cpu-baseline 0 --spinup-ms 0 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python scripts/snap_timeline.py "$f" 10 > $O/timeline.txt 2>&1
rm -rf $O/trace
head -14 $O/kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
cat $O/timeline.txt
