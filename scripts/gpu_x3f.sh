#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv or gdn" > gpurun_out/pytest_x3f.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_x3f.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_x3f.log; exit $rc; }
timeout -k 10 100 python scripts/gdn_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
C=c3_128_2_full,c3_64_3_full,d5_64_3_half,c7_16_2_full
echo "== valu"; timeout -k 10 200 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "== x3 padded N"; FVC_X3_SMALLN=1 timeout -k 10 200 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "== x3 padded N WM1"; FVC_X3_SMALLN=1 FVC_X3_WM=1 timeout -k 10 200 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
