#!/bin/bash
# full GPU suite, then the default bench (A/B over an env knob when AB_VAR is set).
export TMPDIR=/tmp
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for v in ${AB:-x}; do
  env ${AB_VAR:-FVC_NONE}=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench_$v.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('${AB_VAR:-default}=$v', d['value'], r['achieved'], r['ms_per_pframe'], round(sum(v['ms_per_pframe'] for v in d['hbm_kernels'].values()), 3))"
done
