#!/bin/bash
# Round 4: larger rounds into mapped memory -- copied out by a kernel (1, the default) or emitted
# there directly (2) against the header-first copies (0): the round tests under 1 and 2, the rbsr
# line under each, and a trace under 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s18
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run pytest1 600 python -u -m pytest tests/test_rbsr.py -m gpu -q -rf --timeout 300 --timeout-method thread
run pytest2 600 env RSOS_HIP_ROUND_COPYOUT=2 python -u -m pytest tests/test_rbsr.py -m gpu -q -rf --timeout 300 --timeout-method thread
for k in 1 2; do
  run rbsr_m0_$k 300 env RSOS_HIP_ROUND_COPYOUT=0 python3 bench.py --config rbsr
  run rbsr_m1_$k 300 env RSOS_HIP_ROUND_COPYOUT=1 python3 bench.py --config rbsr
  run rbsr_m2_$k 300 env RSOS_HIP_ROUND_COPYOUT=2 python3 bench.py --config rbsr
done
RSOS_HIP_ROUND_COPYOUT=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --config rbsr --steps 3 --warmup 1 > $O/rbsr_trace.log 2>&1 || exit $?
python3 scripts/write_timeline.py $O/tr k_round_bounds > $O/rbsr_timeline_m2.txt 2>&1
rm -rf $O/tr
echo "== done"
