#!/bin/bash
# A/B of x3 launch options selected by environment (e.g. FVC_X3_WS=1): conv_micro per geometry at
# batch 4 for the default and for each "name:VAR=V,VAR2=V2" argument, then the conv parity tests
# under each option.
export TMPDIR=/tmp
TAG=${TAG:-env}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CASES=${CASES:-c3_64_full,c3_64_full_res,c3_128_half,c7_32_64_full,c7_8_32_full,c7_32_16_full,d3_128_half,c3s2_128_half,d5_64_quarter,c3_128_quarter,c1_128_18_full,c3_64_3_full}
run_micro() {
  timeout -k 10 240 env $2 python scripts/conv_micro.py --batch 4 --iters 5 --cases $CASES > $OUT/micro_$1.txt 2>&1 \
    || { cat $OUT/micro_$1.txt; exit 1; }
  echo "== $1 ($2)"; grep -v amdgpu.ids $OUT/micro_$1.txt
}
run_micro base "FVC_X3_NONE=0"
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}; vars=${vars//,/ }
  run_micro $name "$vars"
done
[ -n "$NOTEST" ] && exit 0
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}; vars=${vars//,/ }
  timeout -k 10 400 env $vars python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "conv" > $OUT/pytest_$name.log 2>&1
  rc=$?; echo "pytest $name exit $rc"; grep -E "passed|failed" $OUT/pytest_$name.log | tail -1
  [ $rc -le 1 ] || exit $rc
done
