#!/bin/bash
# Round-1 evidence pass: GPU parity suite, default bench (with CPU baseline), rocprofv3 kernel
# trace/stats of the serial bench, FETCH_SIZE and WRITE_SIZE passes (separate runs).
export TMPDIR=/tmp
O=gpurun_out/${1:-r1r}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log | cut -c1-2500
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --json-out $O/bench_serial_under_rocprof.json > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --serial > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --serial > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
find $O -name "*.csv" | head -20
S=$(find $O/trace -name "run_kernel_stats.csv" | head -1)
F=$(find $O/fetch -name "run_counter_collection.csv" | head -1)
W=$(find $O/write -name "run_counter_collection.csv" | head -1)
python scripts/rocprof_summary.py $S 176 --fetch $F --write $W --json-out $O/x3_traffic.json > $O/summary.txt 2>&1
cat $O/summary.txt
