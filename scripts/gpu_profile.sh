#!/bin/bash
# Profiles for the round: kernel-trace stats + the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the
# bench's workload, and the traffic summary bench.py reads back.  Counters are collected in
# their own runs, never combined with other trace domains.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-config4}
RECORDS=${RECORDS:-100000000}
TAG=${TAG:-r02}
mkdir -p gpurun_out
step() { local name=$1; shift; echo "== $name"; timeout -k 10 600 "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log"; [ $rc -eq 0 ] || exit $rc; }
B="python3 bench.py --config $CONFIG --records $RECORDS --steps 10 --warmup 3 --cpu-baseline 0 --check 0 --e2e 0"
step stats_$CONFIG rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$CONFIG -o run -- $B
step fetch_$CONFIG rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_lift --output-format csv -d gpurun_out/fetch_$CONFIG -o run -- $B
step write_$CONFIG rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_lift --output-format csv -d gpurun_out/write_$CONFIG -o run -- $B
python3 scripts/pmc_traffic.py gpurun_out/fetch_$CONFIG/run_counter_collection.csv gpurun_out/write_$CONFIG/run_counter_collection.csv $CONFIG $RECORDS gpurun_out/${TAG}_traffic_$CONFIG.json
# VALU instruction counts and cycles of the lift kernel (for the VALU roofline)
step valu_$CONFIG rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex k_lift --output-format csv -d gpurun_out/valu_$CONFIG -o run -- $B
python3 scripts/pmc_valu.py gpurun_out/valu_$CONFIG/run_counter_collection.csv gpurun_out/stats_$CONFIG/run_kernel_stats.csv $CONFIG $RECORDS gpurun_out/${TAG}_valu_$CONFIG.json
