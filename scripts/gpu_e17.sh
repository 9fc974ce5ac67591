#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e17; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline --gops-per-gpu 8 --steps 1 --json-out $O/bench_g8.json > $O/bench_g8.log 2>&1 || { tail -20 $O/bench_g8.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_g8.json'));r=d['roofline'];print('G=8',d['value'],d['ms_per_step'],r['achieved'],r['ms_per_pframe'],d['quality'])"
