#!/bin/bash
# stem convs (few input channels, wide outputs: store-bound) under the x3 block-shape knobs, batch 8
export TMPDIR=/tmp
C=c3_6_64_full,c3s2_2_128_full,c5s2_3_64_full
run() { echo "== $1"; env $1 timeout -k 10 120 python scripts/conv_micro.py --cases $C --iters 10 --batch 8 2>&1 | grep -v amdgpu.ids || exit 1; }
run "FVC_NONE=0"
run "FVC_X3_WM=1"
run "FVC_X3_WN=1"
run "FVC_X3_WM=1 FVC_X3_WN=1"
run "FVC_X3_WG=2"
run "FVC_X3_RESERVE=0"
