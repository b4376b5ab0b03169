#!/bin/bash
# Round 4: a peer's round output (mapped page-locked memory) read in by a kernel instead of a copy
# command -- the round tests, then the rbsr line with the kernel read-in on and off, and a trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s21
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run pytest 600 python -u -m pytest tests/test_rbsr.py tests/test_rbsr_latency.py tests/test_bench_path.py -m gpu -q -rf --timeout 300 --timeout-method thread
for k in 1 2; do
  run rbsr_in1_$k 300 python3 bench.py --config rbsr
  run rbsr_in0_$k 300 env RSOS_HIP_ROUND_COPYIN=0 python3 bench.py --config rbsr
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --config rbsr --steps 3 --warmup 1 > $O/rbsr_trace.log 2>&1 || exit $?
python3 scripts/write_timeline.py $O/tr k_round_bounds > $O/rbsr_timeline.txt 2>&1
rm -rf $O/tr
echo "== done"
