#!/bin/bash
# Per-step cost of the RCCL path at the N=8 strong-scaling shard size (100M / 8 = 12.5M records per
# GPU): the plain single-process bench vs torch.distributed.run with one rank (nccl = RCCL), same
# records, same steps.  The difference is what the per-step all_gather + combine + barriers cost.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${N:-12500000}
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29519"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_bench_path.py \
  > gpurun_out/ovh_bench_path.log 2>&1 || { echo "bench path tests failed: $?"; tail -20 gpurun_out/ovh_bench_path.log; exit 1; }
tail -2 gpurun_out/ovh_bench_path.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --config config4 --records $N --steps 40 --warmup 5 --cpu-baseline 0 \
    > gpurun_out/ovh_plain_$i.log 2>&1 || { echo "plain failed: $?"; exit 1; }
  grep -h '"metric"' gpurun_out/ovh_plain_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("plain", d["ms_per_step"], d["roofline"]["achieved"], d["roofline"].get("kernel_avg_us"))'
  timeout -k 10 300 $R bench.py --gpus 1 --config config4 --records $N --steps 40 --warmup 5 --cpu-baseline 0 \
    > gpurun_out/ovh_rccl_$i.log 2>&1 || { echo "rccl failed: $?"; exit 1; }
  grep -h '"metric"' gpurun_out/ovh_rccl_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rccl ", d["ms_per_step"], d["roofline"]["achieved"], d["roofline"].get("kernel_avg_us"))'
done
