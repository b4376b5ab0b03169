#!/bin/bash
# The round's bench logs and kernel-trace summaries: every bench.py workload once, plus the
# rocprofv3 --kernel-trace --stats pass of config2 / config5 / snapshot.  Logs land in
# gpurun_out/logs/ (copied into profiles/ by hand).  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/logs
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 "$O/$name.log" | cut -c1-240; [ $rc -eq 0 ] || exit $rc; }
step bench_config2 300 python bench.py --e2e 1
step bench_config2_100m 300 python bench.py --records 100000000 --steps 10 --warmup 3 --cpu-sample 2000000
step bench_config1 300 python bench.py --config config1
step bench_config3 300 python bench.py --config config3 --steps 10 --cpu-sample 200000
step bench_config5 300 python bench.py --config config5
step bench_config5_overwrite10 300 python bench.py --config config5 --overwrite 0.1 --cpu-baseline 0
step bench_snapshot 300 python bench.py --config snapshot --e2e 1
step bench_u32 300 python bench.py --config bench_u32
for c in config2 config5 snapshot; do
  step stats_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- python3 bench.py --config $c --steps 10 --warmup 3 --cpu-baseline 0 --check 0
done
echo "== done"
