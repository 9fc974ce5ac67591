#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -m gpu -q -p no:cacheprovider --tb=short > gpurun_out/pytest_r1k.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_r1k.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python scripts/conv_micro.py --cases c3_64_full,c3_128_half,d3_128_half,d5_64_quarter,d5_96_64_16 2>&1 | grep -v amdgpu.ids
mkdir -p gpurun_out/prof_r1k
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1k -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --json-out gpurun_out/prof_r1k/bench.json > gpurun_out/prof_r1k/stdout.log 2>&1 || exit $?
python scripts/rocprof_summary.py gpurun_out/prof_r1k/run_kernel_stats.csv 44
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --gops-per-gpu 2 > gpurun_out/bench_g2_r1k.log 2>&1 || exit $?
tail -1 gpurun_out/bench_g2_r1k.log
