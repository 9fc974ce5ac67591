#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv" > gpurun_out/pytest_x3e.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_x3e.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_x3e.log; exit $rc; }
echo "== default"; timeout -k 10 200 python scripts/conv_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== WM=1"; FVC_X3_WM=1 timeout -k 10 200 python scripts/conv_micro.py --cases c3_64_half,c3_128_quarter,c3_128_eighth,d3_128_half,d5_64_quarter,d5_96_64_16 2>&1 | grep -v amdgpu.ids || exit 1
