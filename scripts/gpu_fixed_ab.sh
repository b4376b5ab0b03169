#!/bin/bash
# LDS-staged fixed-length lift (ab/ST) against per-lane loads (ab/NS): parity tests under ST, then
# the encoded probe (fixed path line) alternating, twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fab
mkdir -p $O
RSOS_HIP_TREE=ab/ST timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 240 --timeout-method thread -k "fixed or encoded" \
  > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for v in NS ST; do
  RSOS_HIP_TREE=ab/$v timeout -k 10 200 python3 scripts/encoded_probe.py > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.$rep.log; exit 1; }
  echo "$v.$rep"; grep -h " us " $O/$v.$rep.log | cut -c1-80
done; done
