#!/bin/bash
# A/B of encoded-lift variants built into ab/<v>/rsos_hip (scratch, not tracked): each probe twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in A B C D; do
    RSOS_HIP_TREE=ab/$v timeout -k 10 200 python3 scripts/encoded_probe.py > gpurun_out/ab/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab/$v.$rep.log; exit 1; }
    echo "$v.$rep"; grep -h " us " gpurun_out/ab/$v.$rep.log | cut -c1-70
  done
done
