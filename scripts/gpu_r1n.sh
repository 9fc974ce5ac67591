#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --breakdown > gpurun_out/bench_breakdown_r1n.log 2>&1 || { tail -20 gpurun_out/bench_breakdown_r1n.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_breakdown_r1n.log | cut -c1-200
timeout -k 10 200 python scripts/conv_micro.py > gpurun_out/conv_micro_r1n.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/conv_micro_r1n.log
