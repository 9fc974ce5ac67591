#!/bin/bash
# CU-reserve sweep of the pipelined bench at the 4-GOP default (the reserve leaves CUs of the
# persistent conv grids to the rANS / decode side streams; 40 was tuned at 1 GOP per step).
export TMPDIR=/tmp
O=gpurun_out/reserve
mkdir -p $O
for r in 40 16 24 32 48 64; do
  FVC_PIPELINE_CU_RESERVE=$r timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_r$r.log 2>&1 \
    || { tail -20 $O/bench_r$r.log; exit 1; }
  echo "reserve $r: $(tail -1 $O/bench_r$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
