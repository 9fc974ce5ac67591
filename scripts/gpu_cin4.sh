#!/bin/bash
# cin 2/3 layers on the x3 kernel (FVC_X3_CIN4=1) vs the fp32 kernels: micro, GPU suite, bench A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/cin4
C=c3s2_2_128_full,c5s2_3_64_full
for v in 0 1; do
  FVC_X3_CIN4=$v timeout -k 10 120 python scripts/conv_micro.py --cases $C --iters 20 > gpurun_out/cin4/micro_$v.txt 2>&1 || exit $?
  cat gpurun_out/cin4/micro_$v.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cin4/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/cin4/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/cin4/pytest_gpu.log
for v in 0 1 0 1; do
  FVC_X3_CIN4=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cin4/bench_$v.json 2>gpurun_out/cin4/bench_$v.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/cin4/bench_$v.json').read().strip().splitlines()[-1]); print('cin4=$v', d['value'], d['ms_per_step'])"
done
