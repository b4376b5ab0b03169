#!/bin/bash
# Round 3: config5 at full size (the 100 M test), the encoded bench line, config5 lines (20 / 40 /
# 64 batches) and a kernel trace of 40 batches for the per-kernel breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3_c5
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = 0 ]; then
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_full_size_config5_100m" > $O/test100m.log 2>&1
rc=$?; tail -n 3 $O/test100m.log
if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py --config encoded > $O/encoded.log 2>&1 || { echo "encoded failed"; tail -5 $O/encoded.log; exit 1; }
grep -h '"metric"' $O/encoded.log | cut -c1-400
for k in 20 40 64; do
  timeout -k 10 300 python bench.py --config config5 --steps $k --cpu-baseline 0 > $O/c5_$k.log 2>&1 || { echo "c5 $k failed"; tail -5 $O/c5_$k.log; exit 1; }
  grep -h '"metric"' $O/c5_$k.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- \
  python bench.py --config config5 --steps 40 --warmup 3 --cpu-baseline 0 --spinup-ms 0 > $O/c5t.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python scripts/c5_timeline.py "$f" 10 20 30 > $O/timeline.txt 2>&1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/trace
head -40 $O/kernel_stats.csv | cut -d, -f1-8
