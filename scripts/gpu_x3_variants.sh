#!/bin/bash
# A/B of conv_x3 numerics / schedule variants: per-geometry timing (conv_micro, batch 4 = the
# bench's GOP batch) for the product library and every libfvc_<variant>.so given, then the conv
# parity tests and the 1080p parity tests on each variant.
export TMPDIR=/tmp
TAG=${TAG:-var}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CASES=${CASES:-c3_64_full,c3_64_full_res,c3_128_half,c7_32_64_full,c7_8_32_full,c7_32_16_full,d3_128_half,c3s2_128_half,d5_64_quarter,c3_128_quarter,c1_128_18_full,c3_64_3_full}
for v in base "$@"; do
  if [ "$v" = base ]; then unset FVC_LIB_PATH; else export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$v.so; fi
  echo "== $v"
  timeout -k 10 240 python scripts/conv_micro.py --batch 4 --iters 5 --cases $CASES > $OUT/micro_$v.txt 2>&1 || { cat $OUT/micro_$v.txt; exit 1; }
  cat $OUT/micro_$v.txt
done
[ -n "$NOTEST" ] && exit 0
for v in "$@"; do
  export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$v.so
  timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -m gpu -q -rP --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "conv or 1080p or golden" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v exit $rc"; grep -E "passed|failed" $OUT/pytest_$v.log | tail -2
  grep -E "xscale|1080p flips|parity" $OUT/pytest_$v.log | head -12
  [ $rc -le 1 ] || exit $rc
done
