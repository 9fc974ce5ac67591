#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e15; mkdir -p $O
for cfg in "8 1" "4 2" "8 2"; do set -- $cfg
timeout -k 10 400 python bench.py --no-cpu-baseline --gops-per-gpu $1 --steps $2 --json-out $O/bench_g$1.json > $O/bench_g$1.log 2>&1 || { tail -20 $O/bench_g$1.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_g$1.json'));r=d['roofline'];print('G=$1 steps=$2',d['value'],d['ms_per_step'],r['achieved'],r['ms_per_pframe'],d['quality']['decoder_bitexact'])"
done
