#!/bin/bash
# 32-bit magic-division SpyNet / MC assembly kernels (FVC_ASSEMBLE_Q) vs the 64-bit-index forms:
# kernel tests, then the bench's serial HBM-kernel timings with the switch off and on.
export TMPDIR=/tmp
OUT=gpurun_out/asmq; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do for q in 0 1; do
  FVC_ASSEMBLE_Q=$q timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    --json-out $OUT/b_q${q}_$rep.json > $OUT/b_q${q}_$rep.log 2>&1 || { tail -20 $OUT/b_q${q}_$rep.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/b_q${q}_$rep.json')); h=d['hbm_kernels']
print('q=$q rep $rep', d['value'], {k: (h[k]['ms_per_pframe'], h[k]['gb_per_s']) for k in ('mc_assemble (warp)', 'spynet_assemble (warp)')})"
done; done
