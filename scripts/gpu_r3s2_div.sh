#!/bin/bash
# config5 compaction divisor over long runs (whole compaction cycles): --compact-div D at K batches,
# alternating, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s2div
mkdir -p $O
for rep in 1 2; do for d in ${DIVS:-6 4 3}; do for k in ${STEPS_LIST:-96}; do
  timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --steps $k --compact-div $d > $O/d$d.k$k.$rep.log 2>&1 || { echo "div $d failed"; tail -5 $O/d$d.k$k.$rep.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/d$d.k$k.$rep.log') if l.startswith('{')][0]); print('div $d steps $k rep $rep', d['ms_per_step'], d['value'], 'compactions', d['compactions_in_timed_steps'], 'root', d['root_size'])"
done; done; done
