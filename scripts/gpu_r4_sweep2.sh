#!/bin/bash
# rANS streams per block 128 and GOPs per step 12 / 24 against the defaults (64, 16), reserve 0.
export TMPDIR=/tmp
OUT=gpurun_out/r4sw2; mkdir -p $OUT
run() {  # tag env... args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    $ARGS --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'])"
}
for rep in 1 2; do
  ARGS="" run def_$rep FVC_RANS_SPB_PIPE=64 || exit 1
  ARGS="--gops-per-gpu 24" run g24_$rep FVC_RANS_SPB_PIPE=64 || exit 1
  ARGS="--gops-per-gpu 12" run g12_$rep FVC_RANS_SPB_PIPE=64 || exit 1
done
