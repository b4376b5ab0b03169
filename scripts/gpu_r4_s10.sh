#!/bin/bash
# Round 4: where a device-answered reconciliation's time goes -- bench.py --config rbsr (two 10 M
# replicas, d = 10^4) under a kernel + copy trace, and the line itself.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s10
mkdir -p $O
timeout -k 10 300 python3 bench.py --config rbsr > $O/rbsr.log 2>&1 || exit $?
tail -1 $O/rbsr.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --config rbsr --steps 3 --warmup 1 > $O/rbsr_trace.log 2>&1 || exit $?
python3 scripts/copy_summary.py $O/tr > $O/rbsr_kernels.txt 2>&1
python3 scripts/write_timeline.py $O/tr k_round_bounds > $O/rbsr_timeline.txt 2>&1
rm -rf $O/tr
tail -30 $O/rbsr_kernels.txt
echo "== done"
