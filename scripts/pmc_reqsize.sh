#!/bin/bash
# Read-request size mix and DRAM bytes of the lift (config3's x1.32 over-fetch):
# TCC_EA0_RDREQ_DRAM_32B counts DRAM reads in 32-byte units (a 64-B request = 2, 128-B = 4), so
# x32 gives the HBM read bytes without the FETCH_SIZE width calibration; the 32/64/128-B request
# counts show the widths the access pattern produces.  One counter pass each; the L2 hit rate in
# a third.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "config3 10000000" "config4 100000000"; do
  set -- $spec
  C=$1; R=$2
  B="python3 bench.py --config $C --records $R --steps 5 --warmup 2 --cpu-baseline 0 --check 0 --e2e 0"
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_lift --output-format csv -d gpurun_out/req_$C -o run -- $B > gpurun_out/req_$C.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-include-regex k_lift --output-format csv -d gpurun_out/hit_$C -o run -- $B > gpurun_out/hit_$C.log 2>&1 || exit $?
  python3 scripts/pmc_reqsize.py gpurun_out/req_$C/run_counter_collection.csv gpurun_out/hit_$C/run_counter_collection.csv $C $R gpurun_out/r02_reqsize_$C.json || exit $?
done
