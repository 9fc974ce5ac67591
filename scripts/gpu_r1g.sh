#!/bin/bash
# conv variants A/B (same process per variant), then kernel tests on the default variant
export TMPDIR=/tmp
for v in "FVC_CONV_PIPE=0" "FVC_CONV_PIPE=1" "FVC_CONV_PIPE=1 FVC_CONV_NW=8" "FVC_CONV_PIPE7=1" "FVC_CONV_PIPE7=1 FVC_CONV_NW=8"; do
  echo "== $v"
  env $v timeout -k 10 120 python scripts/conv_micro.py --cases c3_64_full,c3_128_half,c7_32_64_full,c3_128_2_full,d3_128_half || exit $?
done > gpurun_out/micro_r1g.log 2>&1
cat gpurun_out/micro_r1g.log
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --tb=short > gpurun_out/pytest_r1g.log 2>&1
tail -3 gpurun_out/pytest_r1g.log
