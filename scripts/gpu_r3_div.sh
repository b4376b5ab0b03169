#!/bin/bash
# config5 whole-cycle means (64 batches) across compaction divisors, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/div
mkdir -p $O
for rep in 1 2; do
  for d in ${DIVS:-8 6 4 3}; do
    timeout -k 10 300 python bench.py --config config5 --steps ${STEPS:-64} --cpu-baseline 0 --compact-div $d > $O/d$d.$rep.log 2>&1 || { echo "div $d failed"; tail -3 $O/d$d.$rep.log; exit 1; }
    echo "div $d rep $rep $(python3 -c "import json; l=json.loads([x for x in open('$O/d$d.$rep.log') if x.startswith('{')][-1]); print(l['ms_per_step'], l['compactions_in_timed_steps'], l['delta_rows_at_end'])")"
  done
done
