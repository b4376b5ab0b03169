#!/bin/bash
# One GPU session on a gpurun box: named steps, run in order, each under its own time limit;
# the session stops at the first step that fails (a fault, a time limit or a wrong answer: nothing
# more runs on the GPU in that call).  Output goes to gpurun_out/<tag>/<step>.log.
#
#   scripts/gpu_session.sh <tag> <step> [<step> ...]
#
# Steps (env: RECORDS for the profile steps, PYTEST_K for pytest_k, N for the latency steps):
#   pytest            every GPU test
#   pytest_k          the GPU tests matching $PYTEST_K
#   smoke             __graft_entry__.smoke()
#   default config5 config5_40 rbsr snapshot encoded config2 config3
#                     one bench.py line each (the default is configs[3] at N = 1)
#   prof_config4      rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE and VALU passes of the
#                     default line at $RECORDS (100 M unless set), summarised into <tag>_*.json
#   prof_cfg          the same four passes for $CFG at $RECORDS (kernel $KRE, default k_lift),
#                     summarised into <tag>_{traffic,valu}_$CFG.json
#   config3_full      configs[2] at its stated size (100 M x 1 KiB) with its CPU baseline
#   sstore_rounds     sstore_client at 4 / 8 shards, d = 100 / 1, tier on, with per-round times
#   prof_config5      kernel stats + the per-dispatch DRAM byte passes of config5
#   prof_rbsr         kernel stats of the rbsr line
#   latency_tier latency_off
#                     the 1-row write -> d = 1 reconciliation cycle at $N rows (rbsr_latency),
#                     host tier on / off
#   trace_latency_off the same, tier off, under a kernel trace (kernel summary + timeline)
#   latency_phases    the same, tier off, with k_round_tiny's phase clocks (RSOS_HIP_ROUND_DBG=1)
#   latency_host      the same with the host's times per round only (RSOS_HIP_ROUND_DBG=2)
#   sstore_ab         sstore_client with RSOS_HIP_SSTORE_SPIN_US 50 / 300 / 2000, d 1 / 100, tier on / off
#   trace_rbsr        the rbsr line under a kernel + memory-copy trace, its round timeline
#   rbsr_host         the rbsr line with the host's times per large round (RSOS_HIP_ROUND_DBG=2)
#   launch            examples/launch_latency: one waited-for small launch, 16 B and ~2.4 KB arguments
#   interleave_sync interleave_nowait interleave_off
#                     1 M-row batches into both replicas at 10^8 between d = 1 drives (tier_interleave)
#   trace_interleave  the default-policy interleave under a kernel + memory-copy trace
#   trace_interleave_nowait  the same with RSOS_HIP_TIER_SYNC=0
#   trace_interleave_off     the same with the tier off
#   trace_config5     config5 (40 batches) under a kernel trace, four batches' timelines
#   interleave_nowait_ab     interleave_nowait with the foreground stream priority / background CU
#                     mask each on and off (RSOS_HIP_FORE_PRIORITY, RSOS_HIP_BG_RESERVE)
#   sstore            the sharded store's client (examples/sstore_client) on device 0
#   rccl1             every workload under torch.distributed.run with one rank (the nccl = RCCL
#                     process group, its gathers and barriers)
#   inserts           10^6 staged single inserts into 10^5 and 10^7 resident rows (insert_latency)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?usage: gpu_session.sh <tag> <step>...}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
RECORDS=${RECORDS:-100000000}
N=${N:-100000000}
EX=reconcile-rs_amd/examples

run() {  # name, seconds, command...
    local name=$1 t=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 2 "$O/$name.log" | cut -c1-900
    [ $rc -eq 0 ] || exit $rc
}

PMC_B="python3 bench.py --config config4 --records $RECORDS --steps 10 --warmup 3 --cpu-baseline 0 --check 0 --e2e 0"

for step in "$@"; do
    case $step in
    pytest) run pytest 900 python -u -m pytest tests -m gpu -q -rf --maxfail=3 --timeout 300 --timeout-method thread ;;
    pytest_k) run pytest_k 700 python -u -m pytest tests -m gpu -k "${PYTEST_K:?}" -q -rf --maxfail=3 --timeout 300 --timeout-method thread ;;
    smoke) run smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    default) run default 300 python3 bench.py ;;
    config5) run config5 300 python3 bench.py --config config5 ;;
    config5_40) run config5_40 300 python3 bench.py --config config5 --steps 40 ;;
    config5_ab)  # the batch's result block by a kernel store (default) / a copy command, twice each
        for k in 1a 0a 1b 0b; do run config5_ab_$k 300 env RSOS_HIP_COPY_KERNEL=${k%?} python3 bench.py --config config5 --steps 40 --cpu-baseline 0; done ;;
    rbsr) run rbsr 300 python3 bench.py --config rbsr ;;
    trace_rbsr)
        run trace_rbsr 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trrb" -o tr -- python3 bench.py --config rbsr --cpu-baseline 0 --steps 5 --warmup 2
        python3 scripts/write_timeline.py "$O/trrb" k_round_bounds > "$O/${TAG}_rbsr_round_timeline.txt" 2>&1 || true
        cp "$O"/trrb/tr_kernel_stats.csv "$O/${TAG}_rbsr_kernel_stats.csv" 2>/dev/null || true
        rm -f "$O"/trrb/*_trace.csv ;;
    rbsr_copyin_ab)  # a large round's input: copy engine / kernel reading the peer's mapped output
        run rbsr_copyin0 300 env RSOS_HIP_ROUND_COPYIN=0 python3 bench.py --config rbsr --cpu-baseline 0 &&
        run rbsr_copyin1 300 env RSOS_HIP_ROUND_COPYIN=1 python3 bench.py --config rbsr --cpu-baseline 0 &&
        run rbsr_copyin0b 300 env RSOS_HIP_ROUND_COPYIN=0 python3 bench.py --config rbsr --cpu-baseline 0 &&
        run rbsr_copyin1b 300 env RSOS_HIP_ROUND_COPYIN=1 python3 bench.py --config rbsr --cpu-baseline 0 ;;
    rbsr_host) run rbsr_host 300 env RSOS_HIP_ROUND_DBG=2 python3 bench.py --config rbsr --cpu-baseline 0 ;;
    snapshot) run snapshot 300 python3 bench.py --config snapshot ;;
    encoded) run encoded 300 python3 bench.py --config encoded ;;
    config2) run config2 300 python3 bench.py --config config2 ;;
    config3) run config3 300 python3 bench.py --config config3 ;;
    prof_config4)
        R=$RECORDS
        run stats_c4_$R 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_c4_$R" -o run -- $PMC_B
        run fetch_c4_$R 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_lift --output-format csv -d "$O/fetch_c4_$R" -o run -- $PMC_B
        run write_c4_$R 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_lift --output-format csv -d "$O/write_c4_$R" -o run -- $PMC_B
        run valu_c4_$R 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex k_lift --output-format csv -d "$O/valu_c4_$R" -o run -- $PMC_B
        python3 scripts/pmc_traffic.py "$O/fetch_c4_$R/run_counter_collection.csv" "$O/write_c4_$R/run_counter_collection.csv" config4 "$R" "$O/${TAG}_traffic_config4_$R.json" || exit 1
        python3 scripts/pmc_valu.py "$O/valu_c4_$R/run_counter_collection.csv" "$O/stats_c4_$R/run_kernel_stats.csv" config4 "$R" "$O/${TAG}_valu_config4_$R.json" || exit 1
        cp "$O/stats_c4_$R/run_kernel_stats.csv" "$O/${TAG}_config4_${R}_kernel_stats.csv"
        rm -f "$O"/*_c4_$R/*_kernel_trace.csv "$O"/*_c4_$R/*_counter_collection.csv
        ;;
    prof_cfg)  # kernel stats + FETCH_SIZE / WRITE_SIZE + VALU passes of one line: $CFG at $RECORDS
        # (KRE: the kernel profiled, k_lift unless set; k_snap_lift for CFG=snapshot)
        C=${CFG:?} R=$RECORDS K=${KRE:-k_lift}
        B="python3 bench.py --config $C --records $R --steps 10 --warmup 3 --cpu-baseline 0 --check 0 --e2e 0"
        run stats_$C 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_$C" -o run -- $B
        run fetch_$C 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K --output-format csv -d "$O/fetch_$C" -o run -- $B
        run write_$C 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K --output-format csv -d "$O/write_$C" -o run -- $B
        run valu_$C 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex $K --output-format csv -d "$O/valu_$C" -o run -- $B
        python3 scripts/pmc_traffic.py "$O/fetch_$C/run_counter_collection.csv" "$O/write_$C/run_counter_collection.csv" $C "$R" "$O/${TAG}_traffic_$C.json" $K || exit 1
        python3 scripts/pmc_valu.py "$O/valu_$C/run_counter_collection.csv" "$O/stats_$C/run_kernel_stats.csv" $C "$R" "$O/${TAG}_valu_$C.json" $K || exit 1
        cp "$O/stats_$C/run_kernel_stats.csv" "$O/${TAG}_${C}_kernel_stats.csv"
        rm -f "$O"/*_$C/*_kernel_trace.csv "$O"/*_$C/*_counter_collection.csv
        ;;
    sstore_dbg)  # 4 / 8 shards, d = 100, tier on, 3 reps: the sharded rounds' phases and every store's round times
        for g in 4 8; do
            run sstore_dbg_g$g 200 env SSTORE_ROUNDS=1 RSOS_HIP_SSTORE_DBG=1 RSOS_HIP_ROUND_DBG=2 $EX/sstore_client $g 2000000 100 1 3 || exit 1
        done ;;
    sstore_group_ab)  # shards sharing a device: up to 8 / 4 / 2 / 1 shards per thread (RSOS_HIP_SSTORE_GROUP)
        for gr in 8 4 2 1; do
            for g in 4 8; do
                run sstore_grp${gr}_g$g 200 env RSOS_HIP_SSTORE_GROUP=$gr SSTORE_ROUNDS=1 $EX/sstore_client $g 2000000 100 1 20 || exit 1
            done
        done ;;
    sstore_dbg8)  # 8 shards, d = 100, 10 warm reps: the rounds' phases and every store's large-round host times
        run sstore_dbg8 200 env SSTORE_ROUNDS=1 RSOS_HIP_SSTORE_DBG=1 RSOS_HIP_ROUND_DBG=${RDBG:-2} $EX/sstore_client 8 2000000 ${D:-100} 1 10 ;;
    trace_sstore)  # 4 shards, d = 100, 4 reps under a kernel + memory-copy trace (the raw CSVs kept)
        run trace_sstore 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trss" -o tr -- $EX/sstore_client ${SHARDS:-4} 2000000 100 1 4 ;;
    sstore_prio_ab)  # 4 / 8 shards on one device: the stores' streams at high priority (default) / plain
        for pr in 1 0; do
            for g in 4 8; do
                run sstore_prio${pr}_g$g 200 env RSOS_HIP_FORE_PRIORITY=$pr SSTORE_ROUNDS=1 $EX/sstore_client $g 2000000 100 1 20 || exit 1
            done
        done ;;
    config3_full) run config3_full 600 python3 bench.py --config config3_full ;;
    prof_config5)
        run stats_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_c5" -o run -- python3 bench.py --config config5 --cpu-baseline 0
        cp "$O/stats_c5/run_kernel_stats.csv" "$O/${TAG}_config5_kernel_stats.csv"
        rm -f "$O"/stats_c5/*_kernel_trace.csv
        run pmc_c5 600 bash scripts/pmc_c5.sh
        python3 scripts/pmc_c5_summary.py gpurun_out "$O/${TAG}_config5_kernel_stats.csv" "$O/${TAG}_pmc_config5.json" || exit 1
        rm -f gpurun_out/pmc_c5_*/*_counter_collection.csv
        ;;
    prof_rbsr)
        run stats_rbsr 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/stats_rbsr" -o run -- python3 bench.py --config rbsr --cpu-baseline 0
        cp "$O/stats_rbsr/run_kernel_stats.csv" "$O/${TAG}_rbsr_kernel_stats.csv"
        rm -f "$O"/stats_rbsr/*_kernel_trace.csv
        ;;
    latency_tier) run latency_tier 300 $EX/rbsr_latency "$N" 1 200 1 1 ;;
    latency_off) run latency_off 300 $EX/rbsr_latency "$N" 1 40 0 1 ;;
    latency_phases) run latency_phases 300 env RSOS_HIP_ROUND_DBG=1 $EX/rbsr_latency "$N" 1 40 0 1 ;;
    launch) run launch 120 $EX/launch_latency 2000 ;;
    latency_host) run latency_host 300 env RSOS_HIP_ROUND_DBG=2 $EX/rbsr_latency "$N" 1 40 0 1 ;;
    trace_latency_off)
        run trace_latency_off 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trlat" -o tr -- $EX/rbsr_latency "$N" 1 10 0 1
        python3 scripts/write_timeline.py "$O/trlat" k_round > "$O/${TAG}_latency_off_timeline.txt" 2>&1 || true
        cp "$O"/trlat/tr_kernel_stats.csv "$O/${TAG}_latency_off_kernel_stats.csv" 2>/dev/null || true
        rm -rf "$O/trlat"
        ;;
    interleave_sync) run interleave_sync 400 $EX/tier_interleave 100000000 1000000 20 1 c5 2 ;;
    interleave_nowait) run interleave_nowait 400 env RSOS_HIP_TIER_SYNC=0 $EX/tier_interleave 100000000 1000000 12 1 c5 2 3 ;;
    interleave_nowait_ab)  # the foreground priority and background CU mask, each on and off
        run nowait_p0r0 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_FORE_PRIORITY=0 RSOS_HIP_BG_RESERVE=0 RSOS_HIP_STREAM_DBG=1 $EX/tier_interleave 100000000 1000000 8 1 c5 2 &&
        run nowait_p1r0 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_FORE_PRIORITY=1 RSOS_HIP_BG_RESERVE=0 RSOS_HIP_STREAM_DBG=1 $EX/tier_interleave 100000000 1000000 8 1 c5 2 &&
        run nowait_p0r8 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_FORE_PRIORITY=0 RSOS_HIP_BG_RESERVE=8 RSOS_HIP_STREAM_DBG=1 $EX/tier_interleave 100000000 1000000 8 1 c5 2 &&
        run nowait_p0r32 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_FORE_PRIORITY=0 RSOS_HIP_BG_RESERVE=32 RSOS_HIP_STREAM_DBG=1 $EX/tier_interleave 100000000 1000000 8 1 c5 2 ;;
    interleave_nowait_wgs)  # the refresh's background prefix scan on all / 1024 / 256 workgroups
        run nowait_w0 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_BG_PREFIX_WGS=0 $EX/tier_interleave 100000000 1000000 12 1 c5 2 &&
        run nowait_w1024 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_BG_PREFIX_WGS=1024 $EX/tier_interleave 100000000 1000000 12 1 c5 2 &&
        run nowait_w256 300 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_BG_PREFIX_WGS=256 $EX/tier_interleave 100000000 1000000 12 1 c5 2 ;;
    interleave_off) run interleave_off 400 $EX/tier_interleave 100000000 1000000 12 0 c5 2 3 ;;
    trace_nowait_small)  # the no-wait interleave with 3 small cycles after each large batch, under a kernel trace (raw CSVs kept)
        run trace_nowait_small 400 env RSOS_HIP_TIER_SYNC=0 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/trns" -o tr -- $EX/tier_interleave 100000000 1000000 4 1 c5 1 3 ;;
    trace_interleave_nowait)
        run trace_interleave_nowait 400 env RSOS_HIP_TIER_SYNC=0 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trinw" -o tr -- $EX/tier_interleave 100000000 1000000 6 1 c5 1
        python3 scripts/copy_summary.py "$O/trinw" > "$O/${TAG}_interleave_nowait_trace_summary.txt" 2>&1 || true
        python3 scripts/write_timeline.py "$O/trinw" k_cs_minmax > "$O/${TAG}_interleave_nowait_timeline.txt" 2>&1 || true ;;
    nowait_cycles)  # per-cycle write / drive times, and the HIP calls of the same run
        run nowait_cycles 400 env RSOS_HIP_TIER_SYNC=0 TIER_INTERLEAVE_CYCLES=1 RSOS_HIP_ALLOC_DBG=1 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d "$O/nwc" -o tr -- $EX/tier_interleave 100000000 1000000 12 1 c5 2 3
        python3 scripts/long_calls.py "$O/nwc" 5000 > "$O/${TAG}_nowait_long_calls.txt" 2>&1 || true ;;
    nowait_prep_ab)  # the no-wait write waits for its run copy's device preparation (1) or not (0)
        for k in 1a 0a 1b 0b; do run nowait_prep_$k 400 env RSOS_HIP_TIER_SYNC=0 RSOS_HIP_RUN_PREP_WAIT=${k%?} $EX/tier_interleave 100000000 1000000 12 1 c5 2 3; done ;;
    sync_cycles) run sync_cycles 400 env TIER_INTERLEAVE_CYCLES=1 RSOS_HIP_ALLOC_DBG=1 $EX/tier_interleave 100000000 1000000 20 1 c5 2 ;;
    off_cycles) run off_cycles 400 env TIER_INTERLEAVE_CYCLES=1 RSOS_HIP_ALLOC_DBG=1 $EX/tier_interleave 100000000 1000000 12 0 c5 2 3 ;;
    off_drive_trace)  # tier off: per-cycle times and the kernels of each drive (scripts/drive_kernels.py)
        run off_drive_trace 400 env TIER_INTERLEAVE_CYCLES=1 rocprofv3 --kernel-trace --output-format csv -d "$O/odt" -o tr -- $EX/tier_interleave 100000000 1000000 8 0 c5 1
        python3 scripts/drive_kernels.py "$O/odt" "$O/off_drive_trace.log" > "$O/${TAG}_off_drive_kernels.txt" 2>&1 || true ;;
    trace_config5)
        run trace_config5 300 rocprofv3 --kernel-trace --output-format csv -d "$O/c5t" -o c5 -- python3 bench.py --config config5 --steps 40 --cpu-baseline 0
        f=$(find "$O/c5t" -name 'c5_kernel_trace.csv' | head -n 1)
        python3 scripts/c5_timeline.py "$f" 20 21 35 36 > "$O/${TAG}_config5_timeline.txt" 2>&1 || true
        python3 scripts/c5_timeline.py "$f" longest > "$O/${TAG}_config5_compaction_timeline.txt" 2>&1 || true
        rm -f "$f" ;;
    trace_interleave_off)
        run trace_interleave_off 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trio" -o tr -- $EX/tier_interleave 100000000 1000000 6 0 c5 1
        python3 scripts/write_timeline.py "$O/trio" k_cs_minmax > "$O/${TAG}_interleave_off_timeline.txt" 2>&1 || true
        rm -f "$O"/trio/*_trace.csv ;;
    trace_interleave)
        run trace_interleave 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$O/trint" -o tr -- $EX/tier_interleave 100000000 1000000 6 1 c5 1
        python3 scripts/copy_summary.py "$O/trint" > "$O/${TAG}_interleave_trace_summary.txt" 2>&1 || true
        rm -rf "$O/trint"
        ;;
    sstore) run sstore 300 $EX/sstore_client 4 2000000 ;;
    sstore_rounds)  # 4 and 8 shards, d = 100 and 1, tier on: whole drives, aggregates and per-round times
        for g in 4 8; do
            for d in 100 1; do
                run sstore_g${g}_d${d} 200 env SSTORE_ROUNDS=1 $EX/sstore_client $g 2000000 $d 1 20 || exit 1
            done
        done ;;
    sstore_ab)  # the shard threads' spin before sleeping, d = 1 and 100, tier on and off
        for sp in 50 300 2000; do
            for d in 1 100; do
                for t in 1 0; do
                    run sstore_s${sp}_d${d}_t${t} 120 env RSOS_HIP_SSTORE_SPIN_US=$sp $EX/sstore_client 4 2000000 $d $t 10 || exit 1
                done
            done
        done ;;
    rccl1)
        for cfg in config4 config2 config5 snapshot rbsr; do
            extra=""
            [ "$cfg" = config5 ] && extra="--records 20000000"
            run rccl1_$cfg 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
                --master-port 29517 bench.py --gpus 1 --config $cfg --steps 5 --warmup 2 --cpu-baseline 0 $extra
        done
        ;;
    inserts)
        run inserts_1e5 300 $EX/insert_latency 100000 1000000 1
        run inserts_1e7 300 $EX/insert_latency 10000000 1000000 1
        ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== done"
