#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e11; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench$i.json > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench$i.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['achieved'],r['ms_per_pframe'],d['quality'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --json-out $O/bench6.json > $O/bench6.log 2>&1 || { tail -20 $O/bench6.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench6.json'));print('steps6',d['value'],d['ms_per_step'])"
