#!/bin/bash
# upsample-add forms: tests, then bench A/B over FVC_UP2_Q16 (2 = 2x2 blocks, 1 = float4 per thread)
export TMPDIR=/tmp
O=gpurun_out/up2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "upsample" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${AB:-1 2 1 2}; do
  FVC_UP2_Q16=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench_$v.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); h=d['hbm_kernels']
print('up2=$v', d['value'], h['upsample2x_add'], round(sum(v['ms_per_pframe'] for v in h.values()), 3))"
done
