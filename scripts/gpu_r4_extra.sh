#!/bin/bash
# r4 side workloads on the final kernels: tree GOP (LSVC layers), configs[4] 8 views on one GPU,
# configs[3] one rank's 4K GOP-32 share.
export TMPDIR=/tmp
OUT=gpurun_out/r4x; mkdir -p $OUT
run() {  # tag timeout args...
  local tag=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py --cpu-baseline none --no-ref-metrics "$@" --json-out $OUT/$tag.json \
    > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', d['value'], d['unit'], d['ms_per_step'])"
}
run tree 400 --tree --steps 3 --warmup 1 && \
run tree8 400 --tree --gops-per-gpu 8 --steps 3 --warmup 1 && \
run views8 400 --views 8 --steps 3 --warmup 1 && \
run k4_gop32 500 --height 2160 --width 3840 --gop 32 --gops-per-gpu 1 --steps 2 --warmup 1 || exit 1
# two RCCL ranks sharing the box's one GPU (a probe: RCCL may refuse a duplicate device)
echo "== rccl probe"; timeout -k 10 120 python -u scripts/rccl_same_gpu_probe.py 2 > $OUT/rccl_probe.log 2>&1; echo "probe rc=$?"; tail -5 $OUT/rccl_probe.log
