#!/bin/bash
# 128->128 3x3 s1 as four Winograd quarters: tests, micro A/B (FVC_WINO128), bench A/B.
export TMPDIR=/tmp
O=gpurun_out/w128
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_kernels.py -x -v -s --timeout 120 --timeout-method thread -k "wino128 or test_conv" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|of output scale" $O/pytest.log | tail -8
C=c3_128_half,c3_128_quarter,c3_128_eighth
for v in 0 1; do
  FVC_WINO128=$v timeout -k 10 120 python scripts/conv_micro.py --cases $C --iters 10 --batch 8 > $O/micro_$v.txt 2>&1 || exit 1
  echo "wino128=$v"; grep -v amdgpu.ids $O/micro_$v.txt
done
for v in ${AB:-0 1 0 1}; do
  FVC_WINO128=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2>$O/bench_$v.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('wino128=$v', d['value'], r['achieved'], r['ms_per_pframe'], {k: (v['achieved'], v['ms_per_pframe']) for k, v in r['per_kernel'].items()})"
done
