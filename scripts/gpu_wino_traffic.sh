#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of single Winograd geometries (conv_micro, batch 16, one launch timed x 3):
# which side of the traffic exceeds the algorithmic bytes. One counter per rocprofv3 run.
export TMPDIR=/tmp
TAG=${TAG:-wtraf}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CASES=${CASES:-c3_64_full,c3_64_full_res}
for c in ${CASES//,/ }; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/${c}_$ctr -o run -- \
      python3 scripts/conv_micro.py --batch 16 --iters 3 --cases $c > $OUT/${c}_$ctr.log 2>&1 || { tail -5 $OUT/${c}_$ctr.log; exit 1; }
    echo "$c $ctr done"
  done
done
