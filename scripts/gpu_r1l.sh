#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -m gpu -q -p no:cacheprovider --tb=short > gpurun_out/pytest_r1l.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_r1l.log; [ $rc -le 1 ] || exit $rc
for v in "FVC_CONV_BPF=1" "FVC_CONV_BPF=2" "FVC_CONV_BPF=2 FVC_CONV_CC=16"; do
  echo "== $v"; env $v timeout -k 10 120 python scripts/conv_micro.py --cases c3_64_full,c3_128_half,c7_32_64_full,d3_128_half 2>&1 | grep -v amdgpu.ids || exit 1
done
mkdir -p gpurun_out/prof_r1l
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1l -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --json-out gpurun_out/prof_r1l/bench.json > gpurun_out/prof_r1l/stdout.log 2>&1 || exit $?
python scripts/rocprof_summary.py gpurun_out/prof_r1l/run_kernel_stats.csv 44
for g in 2 4; do
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --gops-per-gpu $g > gpurun_out/bench_g${g}_r1l.log 2>&1 || exit $?
tail -1 gpurun_out/bench_g${g}_r1l.log | cut -c1-400
done
