#!/bin/bash
# GPU A/B of an environment switch: selected -m gpu tests, then the default pipelined bench with
# the switch off and on (same process tree, back to back). Usage: gpu_ab_env.sh TAG VAR "tests"
export TMPDIR=/tmp
TAG=$1; VAR=$2; TESTS=${3:-tests}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  --tb=short > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --json-out gpurun_out/bench_${TAG}_$v.json > gpurun_out/bench_${TAG}_$v.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$v.json'));print('$VAR=$v', d['value'], d['roofline']['achieved'])"
done
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --breakdown > gpurun_out/breakdown_$TAG.log 2>&1
