#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 100 python scripts/conv_micro.py --cases c1_128_18_full,c1_64_27_full,c1_64_75_half,c3_128_2_full,c3_64_3_full,d5_64_3_half 2>&1 | grep -v amdgpu.ids || exit 1
for cc in 8 16 32; do echo "CC=$cc"; FVC_X3_CC=$cc timeout -k 10 100 python scripts/conv_micro.py --cases c1_128_18_full,c1_64_27_full,c1_64_75_half 2>&1 | grep -v amdgpu.ids || exit 1; done
echo WN1; FVC_X3_WN=1 timeout -k 10 100 python scripts/conv_micro.py --cases c1_64_75_half 2>&1 | grep -v amdgpu.ids
