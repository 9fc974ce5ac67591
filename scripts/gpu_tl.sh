#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/tl/stdout.log 2>&1 || { tail -5 gpurun_out/tl/stdout.log; exit 1; }
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python scripts/timeline.py $f 0.25 0.62
