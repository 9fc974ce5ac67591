#!/bin/bash
# kernel tests, then the round's rocprofv3 profile set on the final tree
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4p/pytest_kernels.log 2>&1 || { tail -30 gpurun_out/r4p/pytest_kernels.log; exit 1; }
tail -1 gpurun_out/r4p/pytest_kernels.log
bash scripts/gpu_profile_round.sh r4 > gpurun_out/r4p/profile.log 2>&1 || { tail -20 gpurun_out/r4p/profile.log; exit 1; }
tail -2 gpurun_out/r4p/profile.log
