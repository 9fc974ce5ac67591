#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e12; mkdir -p $O
for r in 16 40 64; do
FVC_PIPELINE_CU_RESERVE=$r timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench$r.json > $O/bench$r.log 2>&1 || { tail -20 $O/bench$r.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench$r.json'));r=d['roofline'];print('reserve $r',d['value'],d['ms_per_step'],r['ms_per_pframe'])"
done
