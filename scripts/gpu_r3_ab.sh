#!/bin/bash
# Round 3 A/B of store builds: ab/A (baseline tree) against the working tree, config5 at 40 batches,
# alternating, after the store parity tests on the working tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = 0 ]; then
timeout -k 10 900 python -u -m pytest -x -q -rf --timeout 600 --timeout-method thread -m gpu \
  -k "store or full_size_config5 or host_tier or reference_mirrors or rbsr" tests/ > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E " $O/tests.log | head; exit $rc; fi
fi
for rep in 1 2 3; do
  for v in A B; do
    tree=ab/A/reconcile-rs_amd; [ $v = B ] && tree=reconcile-rs_amd
    RSOS_HIP_TREE=$tree timeout -k 10 300 python bench.py --config config5 --steps ${STEPS:-40} --cpu-baseline 0 > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.$rep.log; exit 1; }
    echo "$v.$rep $(python3 -c "import json,sys; l=json.loads([x for x in open('$O/$v.$rep.log') if x.startswith('{')][-1]); print(l['ms_per_step'], l['compactions_in_timed_steps'])")"
  done
done
