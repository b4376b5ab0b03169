#!/bin/bash
# Round 3: encoded / fixed-length lift parity and A/B, and config5's routed multi-rank rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r3_enc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_fixed_length_records" "tests/test_gpu_parity.py::test_encoded_rows_lift_equals_schema_kernel" \
  "tests/test_gpu_parity.py::test_fixed_equals_encoded_full_size" tests/test_emap.py \
  "tests/test_bench_path.py::test_config5_routed_batches_equal_one_store" > $O/tests.log 2>&1
rc=$?; tail -n 5 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/encoded_r3_probe.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
