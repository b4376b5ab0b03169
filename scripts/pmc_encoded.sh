#!/bin/bash
# Counters for the generic encoded-bytes lift (scripts/encoded_probe.py): kernel-trace stats, then
# one PMC pass of the issue / wait mix (SQ_* in quad-cycles) plus GRBM_GUI_ACTIVE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_enc
mkdir -p $O
timeout -k 10 300 python3 scripts/encoded_probe.py > $O/probe.log 2>&1 || { echo "probe failed"; tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 scripts/encoded_probe.py \
  > $O/stats.log 2>&1 || { echo "stats failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex 'k_lift' --output-format csv -d $O/pmc -o run -- \
  python3 scripts/encoded_probe.py > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
echo done
