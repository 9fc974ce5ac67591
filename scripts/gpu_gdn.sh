#!/bin/bash
# split-precision GDN kernel: GPU tests, then bench A/B (FVC_GDN_X3=0/1) with the hbm_kernels rates.
export TMPDIR=/tmp
O=gpurun_out/gdn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "gdn" -s > $O/pytest_gdn.log 2>&1 || { tail -40 $O/pytest_gdn.log; exit 1; }
grep -E "passed|failed|of scale" $O/pytest_gdn.log | tail -20
for v in ${AB:-0 1 0 1}; do
  FVC_GDN_X3=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench_$v.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); h=d['hbm_kernels']
print('gdn_x3=$v', d['value'], {k: (h[k]['gb_per_s'], h[k]['ms_per_pframe']) for k in ('gdn', 'gdn+tap')}, round(sum(v['ms_per_pframe'] for v in h.values()), 3))"
done
