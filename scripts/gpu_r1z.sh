#!/bin/bash
# Re-entry check of the restored tree: GPU parity suite, smoke, default bench line, rocprof stats.
export TMPDIR=/tmp
O=gpurun_out/r1z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 1 --warmup 1 \
  --no-cpu-baseline --serial > $O/bench_serial_rocprof.log 2>&1 || { tail -20 $O/bench_serial_rocprof.log; exit 1; }
tail -1 $O/bench_serial_rocprof.log
