#!/bin/bash
# Round 4: copy rates of round-sized buffers (microbench/pcie_copy), then larger rounds copied out
# by a kernel into mapped memory (no header round trip): the round tests and the rbsr line with
# the copy-out on and off, and a trace of the line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s17
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "$O/$name.log" | cut -c1-700
  [ $rc -eq 0 ] || exit $rc
}
run pcie 120 microbench/pcie_copy
run pytest 600 python -u -m pytest tests/test_rbsr.py tests/test_rbsr_latency.py tests/test_bench_path.py -m gpu -q -rf --timeout 300 --timeout-method thread
run rbsr_on 300 python3 bench.py --config rbsr
run rbsr_off 300 env RSOS_HIP_ROUND_COPYOUT=0 python3 bench.py --config rbsr
run rbsr_on2 300 python3 bench.py --config rbsr
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --config rbsr --steps 3 --warmup 1 > $O/rbsr_trace.log 2>&1 || exit $?
python3 scripts/write_timeline.py $O/tr k_round_bounds > $O/rbsr_timeline.txt 2>&1
rm -rf $O/tr
echo "== done"
