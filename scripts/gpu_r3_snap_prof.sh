#!/bin/bash
# Round 3 snapshot-reload profiles: kernel-trace stats, the FETCH_SIZE / WRITE_SIZE passes and the
# VALU pass over the fused pass k_snap_lift (each counter group its own run), the summaries
# bench.py reads back, then the bench line that carries them
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/snap_prof
mkdir -p $O
N=10000000
step() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "$O/$name.log"; [ $rc -eq 0 ] || exit $rc; }
B="python3 bench.py --config snapshot --steps 6 --warmup 2 --cpu-baseline 0 --spinup-ms 0"
step stats rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B
step fetch rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_snap_lift --output-format csv -d $O/fetch -o run -- $B
step write rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_snap_lift --output-format csv -d $O/write -o run -- $B
python3 scripts/pmc_traffic.py $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv snapshot $N $O/r03_traffic_snapshot.json k_snap_lift
step valu rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex k_snap_lift --output-format csv -d $O/valu -o run -- $B
python3 scripts/pmc_valu.py $O/valu/run_counter_collection.csv $O/stats/run_kernel_stats.csv snapshot $N $O/r03_valu_snapshot.json k_snap_lift
cp $O/r03_traffic_snapshot.json $O/r03_valu_snapshot.json profiles/
step bench python3 bench.py --config snapshot
grep -h '"metric"' $O/bench.log | cut -c1-2000
rm -rf $O/fetch $O/write $O/valu
