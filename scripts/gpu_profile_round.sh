#!/bin/bash
# Round profile set (committed under profiles/<round>/): rocprofv3 kernel-trace + stats of the
# serial bench (per-kernel time per P-frame), then one FETCH_SIZE and one WRITE_SIZE PMC pass over
# the same command (separate runs, counters only), summarised by scripts/rocprof_summary.py into
# x3_traffic.json (HBM bytes per conv_x3_kernel launch, FETCH_SIZE doubled for gfx950).
export TMPDIR=/tmp
RND=${1:-r2}
OUT=gpurun_out/prof_$RND
mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ref-metrics --serial"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD \
  --json-out $OUT/bench_serial.json > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
echo "stats done"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ref-metrics --serial > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
echo "fetch done"
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ref-metrics --serial > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
echo "write done"
find $OUT -name "*.csv" | head -20
