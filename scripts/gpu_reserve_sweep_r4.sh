#!/bin/bash
# CU reserve for the coder streams (gop.PIPELINE_CU_RESERVE) re-swept with the segment framing
# (shorter rANS chains): bench at the default 16 GOPs, 2 timed steps, alternating.
export TMPDIR=/tmp
OUT=gpurun_out/r4res; mkdir -p $OUT
for rep in 1 2; do for r in 32 16 8 0; do
  FVC_PIPELINE_CU_RESERVE=$r timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    --json-out $OUT/res${r}_$rep.json > $OUT/res${r}_$rep.log 2>&1 || { tail -20 $OUT/res${r}_$rep.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/res${r}_$rep.json')); print('reserve $r rep $rep', d['value'])"
done; done
