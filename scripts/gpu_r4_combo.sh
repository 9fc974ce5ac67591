#!/bin/bash
# Winograd deferred-store A/B (experiment libraries), then the round milestone (scripts/gpu_r4_round.sh).
export TMPDIR=/tmp
mkdir -p gpurun_out/r4m
TAG=r4m/wds VARS="cur ds1 ds2" bash scripts/gpu_wino_variants.sh > gpurun_out/r4m/wds.txt 2>&1 || { tail -30 gpurun_out/r4m/wds.txt; exit 1; }
grep -v amdgpu gpurun_out/r4m/wds.txt | tail -24
bash scripts/gpu_r4_round.sh
