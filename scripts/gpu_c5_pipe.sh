#!/bin/bash
# config5 pipelined multi-batch apply: its parity test + the store tests, then the bench line
# with and without the pipeline at 20 and 40 batches, and a kernel trace of the pipelined line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 240 --timeout-method thread -k "store or many" \
  > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for p in 1 0; do for k in 20 40; do
  timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --pipeline $p --steps $k > $O/c5_p${p}_$k.log 2>&1 || { echo "bench p$p $k failed"; tail -3 $O/c5_p${p}_$k.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/c5_p${p}_$k.log') if l.startswith('{')][0]); print('pipeline $p steps $k', d['ms_per_step'], d['value'], d['compactions_in_timed_steps'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 bench.py --config config5 --cpu-baseline 0 \
  > $O/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
