#!/bin/bash
export TMPDIR=/tmp
C=c3_128_half,c3_128_quarter,d3_128_half,c3s2_128_half
echo default; timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "WM1 WN4"; FVC_X3_WM=1 FVC_X3_WN=4 timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "WM1 WN2"; FVC_X3_WM=1 FVC_X3_WN=2 timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
