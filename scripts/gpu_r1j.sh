#!/bin/bash
export TMPDIR=/tmp
for v in "FVC_CONV_X=0" "FVC_CONV_WN1=1" "FVC_DECONV_FUSED=0" "FVC_DECONV_FUSED=0 FVC_CONV_WN2=1" "FVC_DECONV_FUSED=0 FVC_CONV_WN1=1" "FVC_DECONV_FUSED=0 FVC_CONV_CC=16"; do
  echo "== $v"
  env $v timeout -k 10 120 python scripts/conv_micro.py --cases d3_128_half,d5_64_quarter,d5_96_64_16 || exit $?
done 2>&1 | grep -v amdgpu.ids > gpurun_out/micro_r1j.log
cat gpurun_out/micro_r1j.log
