#!/bin/bash
# One GPU round trip: the full -m gpu suite (one pytest process), then the default bench with its
# CPU leg and parity block. Each GPU step has its own time limit; a failed step ends the script.
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rP \
  --tb=short > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu_$TAG.log
grep -E "passed|failed|error" gpurun_out/pytest_gpu_$TAG.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --json-out gpurun_out/bench_$TAG.json > gpurun_out/bench_$TAG.log 2>&1
rc2=$?
echo "bench exit $rc2"; tail -c 600 gpurun_out/bench_$TAG.log
exit $(( rc > rc2 ? rc : rc2 ))
