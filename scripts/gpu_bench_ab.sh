#!/bin/bash
# Pipelined bench A/B of libfvc builds: each argument is a variant suffix ("base" = libfvc.so);
# runs bench.py (no CPU leg) per library, twice in alternation, and prints value lines.
export TMPDIR=/tmp
TAG=${TAG:-bab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
STEPS=${STEPS:-6}
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset FVC_LIB_PATH; else export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$v.so; fi
    timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --json-out $OUT/bench_${v}_$rep.json \
      > $OUT/bench_${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_${v}_$rep.log; exit 1; }
    python -c "import json;d=json.load(open('$OUT/bench_${v}_$rep.json'));print('$v rep$rep', d['value'], 'x3', d['roofline']['achieved'], d['roofline']['avg_launch_us'])"
  done
done
