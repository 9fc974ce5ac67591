#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step']);print(json.dumps(d['hbm_kernels'],indent=0));print(d['cpu_baseline'])"
