#!/bin/bash
# kernel statistics of config5 (40 batches) for ab/A and the working tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/tab
mkdir -p $O
export TMPDIR=/tmp
for v in A B; do
  tree=ab/A/reconcile-rs_amd; [ $v = B ] && tree=reconcile-rs_amd
  RSOS_HIP_TREE=$tree timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o c5 -- \
    python bench.py --config config5 --steps 40 --warmup 3 --cpu-baseline 0 ${EXTRA:-} > $O/$v.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.log; exit 1; }
  f=$(find $O/t$v -name "*kernel_stats.csv" | head -1); cp "$f" $O/stats_$v.csv
  f=$(find $O/t$v -name "*kernel_trace.csv" | head -1); python3 scripts/c5_timeline.py "$f" 12 13 14 > $O/timeline_$v.txt 2>&1
  rm -rf $O/t$v
  python3 - "$O/stats_$v.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "at::native" in n: continue
    if int(r["TotalDurationNs"]) < 300000: continue
    print(f'{n[:48]:48s} {int(r["Calls"]):5d} {int(r["TotalDurationNs"])/1e3:9.1f} us  avg {int(r["TotalDurationNs"])/int(r["Calls"])/1e3:8.1f}')
PY
done
