#!/bin/bash
export TMPDIR=/tmp
for v in "FVC_CONV_X=0" "FVC_CONV_PIPE=1 FVC_CONV_NW=4 FVC_CONV_CC=16" "FVC_CONV_PIPE=1 FVC_CONV_NW=4 FVC_CONV_CC=8" "FVC_CONV_CC=16" "FVC_CONV_PIPE7=1 FVC_CONV_NW=4 FVC_CONV_CC=8" "FVC_CONV_PIPE=1 FVC_CONV_NW=8 FVC_CONV_CC=8"; do
  echo "== $v"
  env $v timeout -k 10 120 python scripts/conv_micro.py --cases c3_64_full,c3_128_half,c7_32_64_full || exit $?
done > gpurun_out/micro_r1i.log 2>&1
cat gpurun_out/micro_r1i.log | grep -v amdgpu.ids
# serial kernel-trace profile of the whole bench (coder/elementwise breakdown)
mkdir -p gpurun_out/prof_r1i
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1i -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --json-out gpurun_out/prof_r1i/bench.json > gpurun_out/prof_r1i/stdout.log 2>&1 || exit $?
python scripts/rocprof_summary.py gpurun_out/prof_r1i/run_kernel_stats.csv 44
