#!/bin/bash
# x3 config sweep on the main conv geometries (env overrides: FVC_X3_CC / FVC_X3_BLDS / FVC_X3_WM)
export TMPDIR=/tmp
CASES=${CASES:-c3_64_full,c3_64_full_res,c3_128_half,c3_64_half,c3_128_quarter,d3_128_half,c7_32_64_full,c7_32_16_full,d5_64_quarter}
for cfg in "FVC_X3_CC=32" "FVC_X3_CC=16" "FVC_X3_CC=16 FVC_X3_BLDS=0" "FVC_X3_CC=8"; do
  echo "== $cfg"
  env $cfg timeout -k 10 90 python scripts/conv_micro.py --cases $CASES 2>&1 | grep -v amdgpu.ids || exit 1
done
