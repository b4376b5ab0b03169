#!/bin/bash
# store kernels changed: the store / batch parity tests, then the config5 line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fmap.py tests/test_rbsr.py -q -x --timeout 240 --timeout-method thread \
  > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 20 40; do
  timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --steps $k > $O/c5_$k.log 2>&1 || { echo "c5 $k failed"; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/c5_$k.log') if l.startswith('{')][0]); print('steps $k', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c5 -- python3 bench.py --config config5 --cpu-baseline 0 \
  > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
