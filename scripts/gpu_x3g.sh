#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 60 --timeout-method thread -k "conv" > gpurun_out/pytest_x3g.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_x3g.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_x3g.log; exit $rc; }
C=c3_64_full,c3_128_half,c7_32_64_full,d3_128_half,c3_64_half,c3_128_quarter,c7_32_16_full,c3_64_3_full
echo "== single"; timeout -k 10 200 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "== dual"; FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_dual.so timeout -k 10 200 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
