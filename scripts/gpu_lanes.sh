#!/bin/bash
# GOP batch split into concurrent pipeline lanes (FVC_PIPE_LANES) vs one pipeline
export TMPDIR=/tmp
OUT=gpurun_out/lanes; mkdir -p $OUT
run() {  # tag lanes extra-args
  local tag=$1 l=$2; shift 2
  FVC_PIPE_LANES=$l timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    "$@" --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['quality']['decoder_bitexact'], d['quality']['overflow_recomputes'])"
}
for rep in 1 2; do
  run l1_$rep 1 || exit 1
  run l2_$rep 2 || exit 1
  run l2g24_$rep 2 --gops-per-gpu 24 || exit 1
done
