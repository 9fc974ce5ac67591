#!/bin/bash
# Round-1 GPU pass: parity tests, smoke, default bench (with CPU baseline), rocprof kernel stats.
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r1m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1m.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r1m.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r1m.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r1m.log 2>&1 || { tail -20 gpurun_out/smoke_r1m.log; exit 1; }
tail -1 gpurun_out/smoke_r1m.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r1m.log 2>&1 || { tail -20 gpurun_out/bench_r1m.log; exit 1; }
tail -1 gpurun_out/bench_r1m.log | cut -c1-3000
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1m -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --json-out gpurun_out/prof_r1m/bench.json > gpurun_out/prof_r1m/stdout.log 2>&1 || { tail -20 gpurun_out/prof_r1m/stdout.log; exit 1; }
find gpurun_out/prof_r1m -name "*kernel_stats.csv"
