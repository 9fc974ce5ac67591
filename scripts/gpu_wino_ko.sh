#!/bin/bash
# conv_wino_kernel knock-out table on the current kernel (r6): conv_micro at the bench's batch (16)
# for the product library and each libfvc_wko<bits>.so (-D FVC_WINO_KO=<bits>, results wrong by
# construction), then the product again (order check).
export TMPDIR=/tmp
TAG=${TAG:-wko}
OUT=gpurun_out/$TAG; mkdir -p $OUT
CASES=${CASES:-c3_64_full,c3_64_full_relu,c3_64_full_res}
for v in base "$@" base; do
  if [ "$v" = base ]; then unset FVC_LIB_PATH; else export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$v.so; fi
  echo "== $v" | tee -a $OUT/micro.txt
  timeout -k 10 200 python -u scripts/conv_micro.py --batch 16 --iters 5 --cases $CASES >> $OUT/micro.txt 2>&1 || { tail -5 $OUT/micro.txt; exit 1; }
done
cat $OUT/micro.txt
