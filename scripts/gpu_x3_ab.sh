#!/bin/bash
# A/B of conv_x3 builds x launch options: each argument "name:lib:VAR=V,VAR2=V2" (lib = variant
# library suffix or "base" for libfvc.so, vars optional) runs conv_micro at batch 4; then, unless
# NOTEST is set, the conv parity tests under each spec.
export TMPDIR=/tmp
TAG=${TAG:-ab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CASES=${CASES:-c3_64_full,c3_64_full_res,c3_128_half,c7_32_64_full,d3_128_half,c3s2_128_half,c7_32_16_full}
setlib() { if [ "$1" = base ]; then unset FVC_LIB_PATH; else export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$1.so; fi; }
for spec in "$@"; do
  IFS=: read -r name lib vars <<< "$spec"; setlib $lib
  echo "== $name ($lib ${vars})"
  timeout -k 10 240 env ${vars//,/ } python scripts/conv_micro.py --batch 4 --iters 5 --cases $CASES > $OUT/micro_$name.txt 2>&1 \
    || { cat $OUT/micro_$name.txt; exit 1; }
  grep -v amdgpu.ids $OUT/micro_$name.txt
done
[ -n "$NOTEST" ] && exit 0
for spec in "$@"; do
  IFS=: read -r name lib vars <<< "$spec"; setlib $lib
  timeout -k 10 400 env ${vars//,/ } python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "conv" > $OUT/pytest_$name.log 2>&1
  rc=$?; echo "pytest $name exit $rc"; grep -E "passed|failed" $OUT/pytest_$name.log | tail -1
  [ $rc -le 1 ] || exit $rc
done
