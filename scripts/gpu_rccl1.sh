#!/bin/bash
# The RCCL code path of bench.py on one GPU: torch.distributed.run with one rank initialises the
# nccl (RCCL) process group, so init, the per-step all_gather, the barriers and the max-over-ranks
# all_reduce all run -- the multi-GPU path short of the xGMI links.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517"
for cfg in config4 config2 config5 snapshot rbsr; do
  extra=""
  [ "$cfg" = config5 ] && extra="--records 20000000"
  timeout -k 10 300 $R bench.py --gpus 1 --config $cfg --steps 5 --warmup 2 --cpu-baseline 0 $extra \
    > gpurun_out/rccl1_$cfg.log 2>&1 || { echo "rccl1 $cfg failed: $?"; exit 1; }
  grep -h '"metric"' gpurun_out/rccl1_$cfg.log | cut -c1-160
done
