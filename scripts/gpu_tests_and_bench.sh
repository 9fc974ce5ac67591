#!/bin/bash
# GPU round: kernel parity tests first, then end-to-end tests, then a short bench with breakdown.
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --tb=short > gpurun_out/pytest_gpu_kernels_$TAG.log 2>&1
rc=$?
echo "pytest kernels exit $rc" >> gpurun_out/pytest_gpu_kernels_$TAG.log
tail -15 gpurun_out/pytest_gpu_kernels_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -m pytest tests/test_gpu_forward.py -m gpu -q -p no:cacheprovider --tb=short -v > gpurun_out/pytest_gpu_forward_$TAG.log 2>&1
rc=$?
echo "pytest forward exit $rc" >> gpurun_out/pytest_gpu_forward_$TAG.log
tail -30 gpurun_out/pytest_gpu_forward_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --breakdown > gpurun_out/bench_$TAG.log 2>&1
echo "bench exit $?"; tail -3 gpurun_out/bench_$TAG.log
