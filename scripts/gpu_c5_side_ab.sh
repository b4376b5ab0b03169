#!/bin/bash
# A/B of two builds of the store (ab/S: next lift on the same stream, ab/X: on a low-priority side
# stream): the apply_device_many parity test under X, then config5 at 20 and 40 batches, twice each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sab
mkdir -p $O
RSOS_HIP_TREE=ab/X timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 240 --timeout-method thread -k "many or lsm or rejects" \
  > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for v in S X; do for k in 20 40; do
  RSOS_HIP_TREE=ab/$v timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --steps $k > $O/$v.$k.$rep.log 2>&1 || { echo "$v $k failed"; tail -3 $O/$v.$k.$rep.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$v.$k.$rep.log') if l.startswith('{')][0]); print('$v steps $k rep $rep', d['ms_per_step'], d['value'])"
done; done; done
