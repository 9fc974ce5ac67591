#!/bin/bash
# r6: the standalone reproducer (scripts/race_repro.hip) over antagonist x victim; logs in gpurun_out/TAG/
TAG=${1:?tag}; ITERS=${2:-400}
OUT=gpurun_out/$TAG
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -Iinclude scripts/race_repro.hip -o $OUT/race_repro \
  -Lfastvideocodec_amd -l:libfvc_k7.so -Wl,-rpath,$PWD/fastvideocodec_amd || exit 1
for a in ${ANTS:-0 1 2 3}; do
  for v in ${VICTIMS:-0 1 2}; do
    timeout -k 10 120 $OUT/race_repro $ITERS $a $v > $OUT/a${a}_v${v}.log 2>&1
    rc=$?
    grep RESULT $OUT/a${a}_v${v}.log || tail -3 $OUT/a${a}_v${v}.log
    if [ $rc -ne 0 ]; then echo "[repro] a=$a v=$v failed (exit $rc)"; exit $rc; fi
  done
done
