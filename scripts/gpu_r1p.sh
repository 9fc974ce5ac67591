#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1p.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r1p.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r1p.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1p.log 2>&1 || { tail -20 gpurun_out/bench_r1p.log; exit 1; }
tail -1 gpurun_out/bench_r1p.log | cut -c1-400
mkdir -p gpurun_out/prof_r1p
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1p -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial > gpurun_out/prof_r1p/stdout.log 2>&1 || { tail -20 gpurun_out/prof_r1p/stdout.log; exit 1; }
python scripts/rocprof_summary.py gpurun_out/prof_r1p/run_kernel_stats.csv 44
