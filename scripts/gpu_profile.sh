#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (per-kernel durations).
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python bench.py --steps 1 --warmup 1 --no-cpu-baseline --breakdown --json-out $OUT/bench.json > $OUT/bench_stdout.log 2>&1
rc=$?
echo "rocprof exit $rc"
find $OUT -name "*stats*" | head
exit $rc
