#!/bin/bash
# A/B of two store builds in ab/<v> (scratch): config5 at 40 batches, alternating, three times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c5ab
mkdir -p $O
for rep in 1 2 3; do for v in ${VARIANTS:-N T}; do
  RSOS_HIP_TREE=ab/$v timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --steps 40 > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.$rep.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$v.$rep.log') if l.startswith('{')][0]); print('$v rep $rep', d['ms_per_step'], d['value'])"
done; done
