#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -m gpu -q -p no:cacheprovider --tb=short > gpurun_out/pytest_r1f.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r1f.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/conv_micro.py > gpurun_out/micro_r1f.log 2>&1 || exit $?
cat gpurun_out/micro_r1f.log
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown --serial > gpurun_out/bench_serial_r1f.log 2>&1 || exit $?
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/bench_serial_r1f.log | head -12
tail -1 gpurun_out/bench_serial_r1f.log
