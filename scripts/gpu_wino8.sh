#!/bin/bash
# Eight-wave Winograd kernel: its GPU tests (FVC_WINO8=1), then conv_micro A/B against the
# four-wave kernel on the 64-channel 3x3 geometries (batch 8).
export TMPDIR=/tmp
TAG=${1:-w8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
FVC_WINO8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -q -x --timeout 120 --timeout-method thread \
  -p no:cacheprovider -rP --tb=short > $OUT/pytest_wino8.log 2>&1 || { tail -40 $OUT/pytest_wino8.log; exit 1; }
tail -1 $OUT/pytest_wino8.log
CASES=c3_64_full,c3_64_full_res,c3_64_full_relu,c3_64_half,c3_64_half_res,c3_64_half_relu
for v in 0 1 0 1; do
  FVC_WINO8=$v timeout -k 10 180 python -u scripts/conv_micro.py --batch 8 --cases $CASES \
    > $OUT/micro_w8_$v.txt 2>&1 || { echo "micro $v failed"; tail -20 $OUT/micro_w8_$v.txt; exit 1; }
  echo "FVC_WINO8=$v"; cat $OUT/micro_w8_$v.txt
done
