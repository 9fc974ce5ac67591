#!/bin/bash
# r4 profile set (kernel trace + stats, FETCH / WRITE passes) and the per-layer breakdown, both on
# the serial bench without the batch-1 figures.
export TMPDIR=/tmp
mkdir -p gpurun_out/r4p
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --serial --breakdown --cpu-baseline none --no-ref-metrics \
  > gpurun_out/r4p/breakdown.txt 2>&1 || { tail -20 gpurun_out/r4p/breakdown.txt; exit 1; }
echo breakdown done
bash scripts/gpu_profile_round.sh r4 > gpurun_out/r4p/profile.log 2>&1 || { tail -20 gpurun_out/r4p/profile.log; exit 1; }
tail -3 gpurun_out/r4p/profile.log
