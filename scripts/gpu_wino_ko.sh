#!/bin/bash
# conv_wino_kernel knock-out: without the item-end wait for the next item's LDS-DMA rows (wrong results)
export TMPDIR=/tmp
C=c3_64_full,c3_64_full_relu,c3_64_half,c3_64_full_res
for L in fastvideocodec_amd/libfvc.so fastvideocodec_amd/libfvc_kowait.so; do
  echo "== $L"; FVC_LIB_PATH=$L timeout -k 10 150 python scripts/conv_micro.py --cases $C --iters 10 --batch 8 2>&1 | grep -v amdgpu.ids || exit 1
done
