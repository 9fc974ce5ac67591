#!/bin/bash
# SpyNet 7x7 full-resolution layers under the x3 tile knobs (batch 8)
export TMPDIR=/tmp
C=c7_32_64_full,c7_64_32_full,c7_32_16_full,c7_8_32_full
run() { echo "== $1"; env $1 timeout -k 10 150 python scripts/conv_micro.py --cases $C --iters 5 --batch 8 2>&1 | grep -v amdgpu.ids || exit 1; }
run "FVC_NONE=0"
run "FVC_X3_CC=8"
run "FVC_X3_CC=32"
run "FVC_X3_WN=1"
run "FVC_X3_WG=2"
run "FVC_X3_WM=1"
