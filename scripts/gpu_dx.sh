#!/bin/bash
# All-classes transposed conv round trip: its GPU tests and the transposed cases of the kernel
# tests, then conv_micro A/B (per-class conv_x3_kernel FVC_DX=0 vs all-classes FVC_DX=1) on the
# deconv geometries, then (arg 2 = bench) the default pipelined bench. Each GPU step has its own limit.
export TMPDIR=/tmp
TAG=${1:-dx}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deconv.py tests/test_gpu_wino.py "tests/test_gpu_kernels.py::test_conv" \
  "tests/test_gpu_kernels.py::test_conv_then_tap_fused" -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -rP --tb=short > gpurun_out/pytest_dx_$TAG.log 2>&1
rc=$?
echo "dx tests exit $rc"; grep -E "passed|failed|error|err " gpurun_out/pytest_dx_$TAG.log | tail -24
[ $rc -eq 0 ] || exit $rc
CASES=d3_128_half,d3_128_quarter,d3_128_eighth,d5_64_quarter,d5_96_64_16
for v in 0 1; do
  FVC_DX=$v timeout -k 10 180 python -u scripts/conv_micro.py --batch 8 --cases $CASES \
    > gpurun_out/micro_dx${v}_$TAG.txt 2>&1 || { echo "micro $v failed"; tail -20 gpurun_out/micro_dx${v}_$TAG.txt; exit 1; }
  echo "FVC_DX=$v"; cat gpurun_out/micro_dx${v}_$TAG.txt
done
if [ "${2:-}" = "bench" ]; then
  timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --json-out gpurun_out/bench_$TAG.json \
    > gpurun_out/bench_$TAG.log 2>&1
  rc2=$?
  echo "bench exit $rc2"; tail -c 400 gpurun_out/bench_$TAG.log
  exit $rc2
fi
