#!/bin/bash
# rANS decode streams per block inside the GOP pipeline (FVC_RANS_SPB_PIPE) with segment framing.
export TMPDIR=/tmp
OUT=gpurun_out/r4spb; mkdir -p $OUT
for rep in 1 2; do for v in 64 32 16; do
  FVC_RANS_SPB_PIPE=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    --json-out $OUT/spb${v}_$rep.json > $OUT/spb${v}_$rep.log 2>&1 || { tail -20 $OUT/spb${v}_$rep.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/spb${v}_$rep.json')); print('spb $v rep $rep', d['value'])"
done; done
