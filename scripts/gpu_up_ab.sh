#!/bin/bash
# A/B of the Winograd kernel's fused upsample-add forms (experiment libraries libfvc_up<v>.so built
# with -D FVC_UP_KO / FVC_UP_FORM): scripts/up_fuse_micro.py per library, product first.
export TMPDIR=/tmp
TAG=${TAG:-upab}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in base "$@"; do
  if [ "$v" = base ]; then unset FVC_LIB_PATH; else export FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$v.so; fi
  echo "== $v" | tee -a $OUT/micro.txt
  timeout -k 10 200 python -u scripts/up_fuse_micro.py --iters 5 >> $OUT/micro.txt 2>&1 || { tail -5 $OUT/micro.txt; exit 1; }
  tail -2 $OUT/micro.txt
done
