#!/bin/bash
# config5 measurements for profiles/: the default bench line (20 batches), 40 batches, 10 %
# overwrites, and a rocprofv3 kernel trace + stats of the default run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5f
B="python bench.py --config config5 --cpu-baseline 0"
timeout -k 10 300 $B > gpurun_out/c5f/bench20.log 2>&1 || { echo "bench20 failed"; exit 1; }
timeout -k 10 300 $B --steps 40 > gpurun_out/c5f/bench40.log 2>&1 || { echo "bench40 failed"; exit 1; }
timeout -k 10 300 $B --overwrite 0.1 > gpurun_out/c5f/bench_ovw.log 2>&1 || { echo "bench ovw failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5f/prof -o c5 -- \
  python3 bench.py --config config5 --cpu-baseline 0 > gpurun_out/c5f/prof.log 2>&1 || { echo "prof failed"; exit 1; }
for f in bench20 bench40 bench_ovw prof; do grep -h '"metric"' gpurun_out/c5f/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["ms_per_step"], d["value"], d.get("compactions_in_timed_steps"))' $f; done
