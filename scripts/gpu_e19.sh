#!/bin/bash
export TMPDIR=/tmp
C=c3_64_full,c3_128_half,c7_32_64_full,d3_128_half,c3_64_full_res,c3_64_half,c7_32_16_full
for i in 1 2; do
echo "new"; timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "base"; FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_base.so timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
done
