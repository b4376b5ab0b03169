cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_rbsr.py tests/test_gpu_parity.py -k "rbsr or range or store or combine" > gpurun_out/rq_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/rbsr_probe.py --cpu-n 0 > gpurun_out/rbsr_probe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rbsr_prof -o rbsr -- python3 -u scripts/rbsr_probe.py --cpu-n 0 --d 100000 > gpurun_out/rbsr_prof.log 2>&1
