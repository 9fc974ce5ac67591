#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1q.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r1q.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r1q.log
timeout -k 10 100 python scripts/gdn_micro.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1q.log 2>&1 || { tail -20 gpurun_out/bench_r1q.log; exit 1; }
tail -1 gpurun_out/bench_r1q.log | cut -c1-1800
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --breakdown > gpurun_out/bench_breakdown_r1q.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bench_breakdown_r1q.log | head -24 | cut -c1-100
