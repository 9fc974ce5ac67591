#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/tl2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl2 -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tl2/stdout.log 2>&1 || { tail -5 gpurun_out/tl2/stdout.log; exit 1; }
f=$(find gpurun_out/tl2 -name "*kernel_trace.csv" | head -1)
python scripts/gop_timeline.py $f
