#!/bin/bash
# r6: the K7-stem warp-gather hazard, one probe run per experiment library (4K GOP-32, overlapped vs
# serial): bash scripts/gpu_race_r6.sh TAG "lib:LOCATE ..." ; logs in gpurun_out/TAG/
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in $1; do
  lib=${spec%%:*}; loc=${spec#*:}
  echo "[race] $lib LOCATE=$loc"
  FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_$lib.so VIEWS=1 LOCATE=$loc TAG=${TAG}_$lib \
    timeout -k 10 420 python -u scripts/pipeline_race_probe.py > $OUT/$lib.log 2>&1
  rc=$?
  grep -vE 'Warning|warn|amdgpu.ids' $OUT/$lib.log | tail -14
  if [ $rc -ne 0 ]; then echo "[race] $lib failed (exit $rc)"; exit $rc; fi
done
echo "[race] done"
