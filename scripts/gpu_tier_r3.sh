#!/bin/bash
# Round 3 host-tier session: the tier / store parity tests, then the write -> round cycle
# (examples/rbsr_latency with write rows) at n = 10^6 and 10^8, and the staged-insert harness
# (examples/insert_latency) at 10^5 and 10^7 resident rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tier_r3
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = 0 ]; then
timeout -k 10 900 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread -m gpu \
  tests/test_insert_latency.py tests/test_rbsr_latency.py tests/test_rbsr.py tests/test_reference_mirrors.py \
  tests/test_fmap.py "tests/test_gpu_parity.py::test_host_tier_equals_device_answers" \
  "tests/test_gpu_parity.py::test_keys_checked_after_staged_rows" > $O/tests.log 2>&1
rc=$?; tail -n 5 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
fi
L=reconcile-rs_amd/examples/rbsr_latency
I=reconcile-rs_amd/examples/insert_latency
for w in 0 1 1000; do
  timeout -k 10 300 $L 1000000 1 300 1 $w >> $O/latency_1e6.jsonl 2>> $O/latency.err || exit $?
done
tail -n 3 $O/latency_1e6.jsonl
for w in 1 1000; do
  timeout -k 10 600 $L 100000000 1 40 1 $w >> $O/latency_1e8.jsonl 2>> $O/latency.err || exit $?
  tail -n 1 $O/latency_1e8.jsonl
done
for n in 100000 10000000; do
  timeout -k 10 300 $I $n 1000000 1 >> $O/insert.jsonl 2>> $O/insert.err || exit $?
  tail -n 1 $O/insert.jsonl
done
