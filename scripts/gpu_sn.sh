#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv" > gpurun_out/pytest_sn.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sn.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_sn.log; exit $rc; }
timeout -k 10 200 python scripts/conv_micro.py --cases c3_128_2_full,c3_64_3_full,d5_64_3_half,c7_16_2_full 2>&1 | grep -v amdgpu.ids || exit 1
