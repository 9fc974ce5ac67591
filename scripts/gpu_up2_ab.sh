#!/bin/bash
# product libfvc.so vs the previous commit's library (experiment
# library libfvc_wold.so from the previous commit): kernel tests, then the bench's serial HBM timings
export TMPDIR=/tmp
OUT=gpurun_out/up2ab; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do for v in old new; do
  if [ $v = old ]; then L="FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_wold.so"; else L="FVC_NONE=0"; fi
  env $L timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --cpu-baseline none --no-ref-metrics \
    --json-out $OUT/b_${v}_$rep.json > $OUT/b_${v}_$rep.log 2>&1 || { tail -20 $OUT/b_${v}_$rep.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/b_${v}_$rep.json')); h=d['hbm_kernels']
print('$v rep $rep', d['value'], {k: (h[k]['ms_per_pframe'], h[k]['gb_per_s']) for k in ('tap_gather', 'gdn+tap', 'upsample2x_add')})"
done; done
