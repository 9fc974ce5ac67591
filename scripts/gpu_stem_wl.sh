#!/bin/bash
# stems (store-bound small-cin convs) with weights staged by LDS-DMA (FVC_X3_WL=1) vs the default,
# and the practical HBM copy / fill / read rates
export TMPDIR=/tmp
OUT=gpurun_out/stemwl; mkdir -p $OUT
C=c3_6_64_full,c3s2_2_128_full,c5s2_3_64_full
timeout -k 10 120 python scripts/copy_peak.py > $OUT/copy_peak.txt 2>&1 || { tail $OUT/copy_peak.txt; exit 1; }
cat $OUT/copy_peak.txt
for rep in 1 2; do for wl in 0 1; do
  FVC_X3_WL=$wl timeout -k 10 180 python -u scripts/conv_micro.py --cases $C --iters 10 --batch 8 > $OUT/wl${wl}_$rep.txt 2>&1 || { tail -20 $OUT/wl${wl}_$rep.txt; exit 1; }
  echo "== WL=$wl rep $rep"; grep -v amdgpu.ids $OUT/wl${wl}_$rep.txt
done; done
