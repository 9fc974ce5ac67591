#!/bin/bash
# rANS decode streams-per-block A/B: coder tests under each value, then rocprofv3 kernel stats of
# the serial bench (k_rans_decode average per launch) for each value.
export TMPDIR=/tmp
OUT=gpurun_out/spb; mkdir -p $OUT
for v in "$@"; do
  FVC_RANS_SPB=$v timeout -k 10 300 python -m pytest tests/test_gpu_coder.py tests/test_gpu_kernels.py -m gpu -q -k "rans or compress or coder" \
    -p no:cacheprovider > $OUT/pt_$v.log 2>&1 || { tail -5 $OUT/pt_$v.log; exit 1; }
  echo "tests spb=$v: $(tail -1 $OUT/pt_$v.log)"
done
for v in "$@"; do
  FVC_RANS_SPB=$v timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$v -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial > $OUT/prof_$v.log 2>&1 || { tail -5 $OUT/prof_$v.log; exit 1; }
  f=$(find $OUT/p$v -name "*kernel_stats.csv" | head -1)
  echo "spb=$v $(grep k_rans_decode $f | cut -d, -f2-4)"
done
