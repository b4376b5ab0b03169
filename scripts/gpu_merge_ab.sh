#!/bin/bash
# wave-searched merge tiles (ab/W) against the one-lane searches (ab/O): store tests under W, then
# config5 at 40 batches alternating, three times, and one kernel trace of each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mab
mkdir -p $O
RSOS_HIP_TREE=ab/W timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fmap.py -q -x --timeout 240 --timeout-method thread -k "store or many or fmap or incremental or batch" \
  > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
VARIANTS="O W" bash scripts/gpu_c5_ab.sh || exit 1
for v in O W; do
  RSOS_HIP_TREE=ab/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o c5 -- python3 bench.py --config config5 --cpu-baseline 0 \
    > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
done
echo done
