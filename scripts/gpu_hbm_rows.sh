#!/bin/bash
# Row-structured upsample-add / avgpool kernels: parity suite, then two default bench lines.
export TMPDIR=/tmp
O=gpurun_out/${1:-rows}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], {k: (v["gb_per_s"], v["ms_per_pframe"]) for k, v in d["hbm_kernels"].items()})'
done
