#!/bin/bash
# Bench in serial mode (clean per-kernel breakdown) and overlapped mode.
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown --serial > gpurun_out/bench_serial_$TAG.log 2>&1 || exit $?
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/bench_serial_$TAG.log | head -40
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --gops-per-gpu 2 > gpurun_out/bench_g2_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_g2_$TAG.log
