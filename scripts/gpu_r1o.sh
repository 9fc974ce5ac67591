#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r1o.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r1o.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r1o.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r1o.log 2>&1 || { tail -20 gpurun_out/smoke_r1o.log; exit 1; }
tail -1 gpurun_out/smoke_r1o.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r1o.log 2>&1 || { tail -20 gpurun_out/bench_r1o.log; exit 1; }
tail -1 gpurun_out/bench_r1o.log | cut -c1-1500
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --breakdown > gpurun_out/bench_breakdown_r1o.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bench_breakdown_r1o.log | head -30 | cut -c1-120
