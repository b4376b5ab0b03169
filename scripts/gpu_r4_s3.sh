#!/bin/bash
# Round 4, third GPU session: config5 after the two-level sort positions -- bench lines (20 and 40
# batches) with the roofline, a kernel-stats trace and the three PMC passes of scripts/pmc_c5.sh,
# summarised into r04_pmc_config5.json; then the default line and smoke.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s3
mkdir -p $O
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc
}
run c5_20 300 python3 bench.py --config config5
run c5_40 300 python3 bench.py --config config5 --steps 40
run c5_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5stats -o run -- python3 bench.py --config config5 --steps 6 --warmup 2 --cpu-baseline 0 --spinup-ms 0
run pmc 500 bash scripts/pmc_c5.sh
S=$(ls $O/c5stats/*/*kernel_stats.csv $O/c5stats/*kernel_stats.csv 2>/dev/null | head -1)
cp "$S" $O/config5_kernel_stats.csv
run pmc_summary 60 python3 scripts/pmc_c5_summary.py gpurun_out $O/config5_kernel_stats.csv $O/r04_pmc_config5.json
rm -rf $O/c5stats
run default 300 python3 bench.py
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
echo "== done"
