#!/bin/bash
# Round 4: tiny rounds over base + pending delta run without copy commands (mapped input and
# output) -- the round tests, the tier-off write -> round cycle at 10^8, the tier-off interleave,
# and the no-wait interleave with 4 and 8 hardware queues (do the refresh copies of one store
# hold up the other store's stream when streams share a queue?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s14
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
}
run pytest 700 python -u -m pytest tests/test_rbsr.py tests/test_rbsr_latency.py tests/test_gpu_parity.py -k "rbsr or round or lsm or select or split or resolve or latency" -m gpu -q -rf --timeout 300 --timeout-method thread
run latency 400 reconcile-rs_amd/examples/rbsr_latency 100000000 1 40 0 1
run interleave_off 400 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 0 c5 2 3
run nowait_q4 400 env RSOS_HIP_TIER_SYNC=0 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
run nowait_q8 400 env RSOS_HIP_TIER_SYNC=0 GPU_MAX_HW_QUEUES=8 reconcile-rs_amd/examples/tier_interleave 100000000 1000000 12 1 c5 2 3
echo "== done"
