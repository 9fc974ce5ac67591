#!/bin/bash
# activation stores with the non-temporal cache policy (libfvc_nt.so, -DFVC_STORE_AUX=2) vs default
export TMPDIR=/tmp
C=c3_64_full,c3_128_half,c7_32_64_full,d3_128_half,c3_6_64_full
for L in fastvideocodec_amd/libfvc.so fastvideocodec_amd/libfvc_nt.so; do
  echo "== $L"; FVC_LIB_PATH=$L timeout -k 10 150 python scripts/conv_micro.py --cases $C --iters 5 --batch 16 2>&1 | grep -v amdgpu.ids || exit 1
done
for L in prod nt prod nt; do
  lib=fastvideocodec_amd/libfvc_$L.so; [ $L = prod ] && lib=fastvideocodec_amd/libfvc.so
  FVC_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/nt_$L.json 2>/dev/null || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/nt_$L.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$L', d['value'], r['achieved'], {k: v['achieved'] for k, v in r['per_kernel'].items()})"
done
