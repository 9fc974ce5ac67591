#!/bin/bash
# Winograd ReLU input applied in place in LDS (product) vs in the transform (libfvc_relutr.so)
export TMPDIR=/tmp
O=gpurun_out/wrelu
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
C=c3_64_full_relu,c3_64_half_relu,c3_64_full,c3_64_full_res
for L in fastvideocodec_amd/libfvc_relutr.so fastvideocodec_amd/libfvc.so; do
  echo "== $L"; FVC_LIB_PATH=$L timeout -k 10 120 python scripts/conv_micro.py --cases $C --iters 10 --batch 8 2>&1 | grep -v amdgpu.ids || exit 1
done
for L in relutr prod relutr prod; do
  lib=fastvideocodec_amd/libfvc_$L.so; [ $L = prod ] && lib=fastvideocodec_amd/libfvc.so
  FVC_LIB_PATH=$lib timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$L.json 2>$O/bench_$L.err || exit $?
  python -c "
import json; d=json.loads(open('$O/bench_$L.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$L', d['value'], r['achieved'], {k: (v['achieved'], v['ms_per_pframe']) for k, v in r['per_kernel'].items()})"
done
