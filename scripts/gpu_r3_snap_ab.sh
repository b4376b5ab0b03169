#!/bin/bash
# Round 3 A/B of the snapshot reload: ab/A against the working tree (bench lines, alternating),
# then PMC passes over k_snap_lift for both builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/snap_ab
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in A B; do
    tree=ab/A/reconcile-rs_amd; [ $v = B ] && tree=reconcile-rs_amd
    RSOS_HIP_TREE=$tree timeout -k 10 300 python bench.py --config snapshot --cpu-baseline 0 > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.$rep.log; exit 1; }
    echo "$v.$rep $(python3 -c "import json,sys; l=json.loads([x for x in open('$O/$v.$rep.log') if x.startswith('{')][-1]); print(l['ms_per_step'])")"
  done
done
B="python3 bench.py --config snapshot --steps 4 --warmup 1 --cpu-baseline 0 --spinup-ms 0"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  for v in A B; do
    tree=ab/A/reconcile-rs_amd; [ $v = B ] && tree=reconcile-rs_amd
    RSOS_HIP_TREE=$tree timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_snap_lift" --output-format csv -d $O/pmc_${v}_$i -o run -- $B \
      > $O/pmc_${v}_$i.log 2>&1 || { echo "pass $v $i failed: $?"; tail -5 $O/pmc_${v}_$i.log; exit 1; }
    f=$(find $O/pmc_${v}_$i -name "*counter_collection.csv" | head -1)
    python3 - "$f" "$v.$i" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[2], {k: round(v / max(1, n[k] / 1), 1) for k, v in sorted(acc.items())}, "dispatches", max(n.values()) if n else 0)
PY
  done
done
