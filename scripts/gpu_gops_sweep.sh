#!/bin/bash
# GOPs-per-step sweep of the default 1080p bench (steps 3, warmup 1); one JSON line per setting.
export TMPDIR=/tmp
mkdir -p gpurun_out/gops_sweep
for g in ${GOPS:-4 6 8}; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --gops-per-gpu $g --no-cpu-baseline \
    > gpurun_out/gops_sweep/g$g.json 2> gpurun_out/gops_sweep/g$g.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/gops_sweep/g$g.json').read().strip().splitlines()[-1]); print($g, d['value'], d['ms_per_step'])"
done
