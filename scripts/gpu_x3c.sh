#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv" > gpurun_out/pytest_x3c.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_x3c.log; [ $rc -eq 0 ] || exit $rc
C=c3_64_full,c3_128_half,c7_32_64_full,d3_128_half,d5_64_quarter,c7_32_16_full
for v in "FVC_CONV_PRECISION=f32" "FVC_X3_NW=8" "FVC_X3_NW=8 FVC_X3_BPC=2" "FVC_X3_NW=4" "FVC_X3_NW=4 FVC_X3_WM=4" "FVC_X3_NW=8 FVC_X3_WM=1" "FVC_X3_CC=32" "FVC_X3_CC=8"; do
  echo "== $v"; env $v timeout -k 10 120 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
done
