#!/bin/bash
# A/B of Winograd kernel variants built as fastvideocodec_amd/libfvc_w<name>.so (experiment
# libraries loaded with FVC_LIB_PATH, never the product): the Winograd tests, then conv_micro on the
# 64-channel 3x3 geometries, every variant twice in alternation.
export TMPDIR=/tmp
TAG=${TAG:-wv}
VARS=${VARS:-base e1 e2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CASES=c3_64_full,c3_64_full_res,c3_64_full_relu,c3_64_half,c3_64_half_res,c3_64_half_relu
for v in $VARS; do
  FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_w$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -q -x \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
for rep in 1 2; do for v in $VARS; do
  FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_w$v.so timeout -k 10 180 python -u scripts/conv_micro.py --batch 8 \
    --cases $CASES > $OUT/micro_${v}_$rep.txt 2>&1 || { tail -20 $OUT/micro_${v}_$rep.txt; exit 1; }
  echo "== $v rep $rep"; grep -v amdgpu.ids $OUT/micro_${v}_$rep.txt
done; done
