#!/bin/bash
# final r4 check after the HBM-kernel changes: whole -m gpu suite, smoke, default bench
export TMPDIR=/tmp
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 420 python -u bench.py --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || { tail -30 $OUT/bench_default.log; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_default.json')); h=d['hbm_kernels']
print('value', d['value'], 'x3frac', d['roofline']['frac_of_x3_ceiling'], 'hbm ms', round(sum(v['ms_per_pframe'] for v in h.values()),3))"
