#!/bin/bash
# round 3, session 2: store-path GPU tests of the in-tree build, then an A/B of config5 (ab/A = the
# previous build, ab/B = this one) at 40 batches, alternating, and a kernel trace of B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s2ab
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" = 0 ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -x -v \
  --timeout 300 --timeout-method thread -m gpu -k "${TESTK:-not nothing}" \
  > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
for rep in $(seq 1 ${REPS:-2}); do for v in ${VARIANTS:-D F G}; do
  # a variant's extra environment: ENV_<v>="NAME=value ..." (e.g. an A/B switch of one build)
  eval "XENV=\${ENV_$v:-}"
  env $XENV RSOS_HIP_TREE=ab/$v timeout -k 10 300 python bench.py --config config5 --cpu-baseline 0 --steps ${STEPS:-40} > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.$rep.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$v.$rep.log') if l.startswith('{')][0]); print('$v rep $rep', d['ms_per_step'], d['value'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- \
  python3 bench.py --config config5 --steps 40 --warmup 3 --cpu-baseline 0 --spinup-ms 0 > $O/c5t.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/c5_timeline.py "$f" 10 20 30 > $O/timeline.txt 2>&1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/trace
head -32 $O/timeline.txt
