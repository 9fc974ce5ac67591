#!/bin/bash
# HIP stream priorities in the GOP pipeline (experiment): encoder chain high / reconstruction high
export TMPDIR=/tmp
OUT=gpurun_out/prio; mkdir -p $OUT
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    --json-out $OUT/$tag.json > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['quality']['decoder_bitexact'])"
}
for rep in 1 2; do
  run def_$rep FVC_NONE=0 || exit 1
  run enc_$rep FVC_PRIO_ENC=-1 || exit 1
  run rec_$rep FVC_PRIO_REC=-1 || exit 1
done
