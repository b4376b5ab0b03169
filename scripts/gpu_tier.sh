#!/bin/bash
# Host-tier session: the tier's parity tests, then the reference's reconciliation_drive through the
# C ABI (examples/rbsr_latency) at n = 10^6 from the device and from the host tier.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu \
  tests/test_rbsr.py tests/test_reference_mirrors.py tests/test_rbsr_latency.py tests/test_snapshot.py \
  "tests/test_gpu_parity.py::test_host_tier_equals_device_answers" > gpurun_out/tier_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/tier_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
for tier in 0 1; do
  for d in 1 100; do
    timeout -k 10 300 reconcile-rs_amd/examples/rbsr_latency 1000000 $d ${REPS:-500} $tier >> gpurun_out/tier_latency.jsonl 2>> gpurun_out/tier_latency.err || exit $?
  done
done
cat gpurun_out/tier_latency.jsonl
