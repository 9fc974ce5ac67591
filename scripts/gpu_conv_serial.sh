#!/bin/bash
# global conv serialisation across streams (FVC_CONV_SERIAL=1) vs the default four-stream overlap
export TMPDIR=/tmp
OUT=gpurun_out/cser; mkdir -p $OUT
for rep in 1 2; do for v in 0 1; do
  FVC_CONV_SERIAL=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    --json-out $OUT/s${v}_$rep.json > $OUT/s${v}_$rep.log 2>&1 || { tail -20 $OUT/s${v}_$rep.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/s${v}_$rep.json')); print('serial=$v rep $rep', d['value'], d['quality']['decoder_bitexact'])"
done; done
