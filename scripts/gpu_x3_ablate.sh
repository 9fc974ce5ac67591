#!/bin/bash
# Ablation of conv_x3_kernel<16,2,2,8,0> on the 3x3 64->64 1080p layer (FVC_X3_DBG bits, see the kernel)
export TMPDIR=/tmp
export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_base.so
export FVC_X3_CC=16 FVC_X3_BLDS=0
for d in 0 4 16 0; do
  echo "== DBG=$d"; FVC_X3_DBG=$d timeout -k 10 100 python scripts/conv_micro.py --cases c3_64_full,c3_64_half 2>&1 | grep -v amdgpu.ids || exit 1
done
