#!/bin/bash
# kernel trace of the pipelined default bench (1 warm-up + 1 timed step, then the serial roofline
# pass) for scripts/gop_timeline.py
export TMPDIR=/tmp
OUT=gpurun_out/tl_r4; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 1 \
  --cpu-baseline none --no-ref-metrics --json-out $OUT/bench.json > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 scripts/gop_timeline.py $f | tee $OUT/timeline.txt
rm -f $f
