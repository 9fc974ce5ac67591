#!/bin/bash
# Winograd kernel round trip: its GPU tests, then conv_micro A/B (direct x3 vs Winograd) on the
# 64-channel 3x3 geometries, then the full round (gpu_round.sh). Each GPU step has its own limit.
export TMPDIR=/tmp
TAG=${1:-wino}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -rP --tb=short > gpurun_out/pytest_wino_$TAG.log 2>&1
rc=$?
echo "wino tests exit $rc"; grep -E "passed|failed|error|err " gpurun_out/pytest_wino_$TAG.log | tail -20
[ $rc -eq 0 ] || exit $rc
CASES=c3_64_full,c3_64_full_res,c3_64_half,c3_64_half_res
for v in 0 1; do
  FVC_WINO=$v timeout -k 10 180 python -u scripts/conv_micro.py --batch 8 --cases $CASES \
    > gpurun_out/micro_wino${v}_$TAG.txt 2>&1 || { echo "micro $v failed"; tail -20 gpurun_out/micro_wino${v}_$TAG.txt; exit 1; }
  echo "FVC_WINO=$v"; cat gpurun_out/micro_wino${v}_$TAG.txt
done
[ "${2:-}" = "full" ] && exec_round=1 || exec_round=0
if [ $exec_round -eq 1 ]; then bash scripts/gpu_round.sh $TAG; fi
