#!/bin/bash
# wino128 per-image gate at the 16-GOP default: micro at batch 16, bench A/B over FVC_WINO128_MINPIX
export TMPDIR=/tmp
C=c3_128_half,c3_128_quarter,c3_128_eighth
for v in "FVC_WINO128=0" "FVC_WINO128_MINPIX=0"; do
  echo "== $v"; env $v timeout -k 10 150 python scripts/conv_micro.py --cases $C --iters 10 --batch 16 2>&1 | grep -v amdgpu.ids || exit 1
done
for m in 200000 100000 200000 100000; do
  FVC_WINO128_MINPIX=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/w128g_$m.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/w128g_$m.json').read().strip().splitlines()[-1]); print('minpix=$m', d['value'])"
done
