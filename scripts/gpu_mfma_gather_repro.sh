#!/bin/bash
# r6: scripts/mfma_gather_repro.hip over antagonist kind / shape and victim loads in flight
TAG=${1:?tag}; ITERS=${2:-200}
OUT=gpurun_out/$TAG; mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/mfma_gather_repro.hip -o $OUT/mfma_gather_repro || exit 1
for spec in ${SPECS:-"4 512 1 8" "0 512 1 8" "1 512 1 8" "2 512 1 8" "3 512 1 8" "1 512 1 4" "1 64 1 8" "1 256 1 8" "1 256 2 8" "1 1024 1 8" "1 64 4 8"}; do
  timeout -k 10 120 $OUT/mfma_gather_repro $ITERS $spec > $OUT/run.log 2>&1
  rc=$?
  grep RESULT $OUT/run.log || tail -3 $OUT/run.log
  if [ $rc -ne 0 ]; then echo "[repro] $spec failed (exit $rc)"; exit $rc; fi
done
