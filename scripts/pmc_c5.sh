#!/bin/bash
# PMC passes over config5's per-batch kernels (sort, searches, merge): DRAM read bytes, L2 hits,
# instruction mix and wave occupancy.  One rocprofv3 pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --config config5 --steps 6 --warmup 2 --cpu-baseline 0 --spinup-ms 0"
RX='k_cs_|k_search_sampled|k_merge_run|k_delta_build|k_lift'
i=0
for grp in "TCC_EA0_RDREQ_DRAM_32B_sum TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_c5_$i -o run -- $B \
    > gpurun_out/pmc_c5_$i.log 2>&1 || { echo "pass $i failed: $?"; tail -5 gpurun_out/pmc_c5_$i.log; exit 1; }
done
echo done
