#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/dbg
timeout -k 10 700 python -u -m pytest -x -q -rf --timeout 600 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_full_size_config5_100m" > gpurun_out/dbg/t.log 2>&1
tail -3 gpurun_out/dbg/t.log; grep -E "^E " gpurun_out/dbg/t.log | head -5
