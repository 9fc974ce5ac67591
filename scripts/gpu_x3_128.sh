#!/bin/bash
# 128->128 3x3 stride-1 layers on conv_x3_kernel: block shapes (2 strips x 2 N-tiles, two N-groups
# vs 1 strip x 4 N-tiles, one N-group = input staged once) and channel chunks, batch 8.
export TMPDIR=/tmp
C=c3_128_half,c3_128_quarter,c3_128_eighth
run() { echo "== $1"; env $1 timeout -k 10 120 python scripts/conv_micro.py --cases $C --iters 10 --batch 8 2>&1 | grep -v amdgpu.ids || exit 1; }
run "FVC_NONE=0"
run "FVC_X3_WM=1 FVC_X3_WN=4"
run "FVC_X3_WM=1 FVC_X3_WN=4 FVC_X3_CC=16"
run "FVC_X3_CC=16"
run "FVC_X3_WM=1 FVC_X3_WN=2"
