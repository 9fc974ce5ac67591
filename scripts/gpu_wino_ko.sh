#!/bin/bash
# Knock-out timing of the Winograd kernel (experiment libraries libfvc_wko<K>.so, FVC_WINO_KO=K:
# results are wrong by construction; conv_micro timings only).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wko}; mkdir -p $OUT
for rep in 1 2; do for k in ${KOS:-0 1 2 3 4 8}; do
  FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_wko$k.so timeout -k 10 120 python -u scripts/conv_micro.py --batch 8 \
    --cases c3_64_full,c3_64_full_relu > $OUT/ko${k}_$rep.txt 2>&1 || { tail -20 $OUT/ko${k}_$rep.txt; exit 1; }
  echo "== KO $k rep $rep"; grep -v amdgpu.ids $OUT/ko${k}_$rep.txt
done; done
