#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e7; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
C=c3_128_2_full,c3_64_3_full,d5_64_3_half,c3_64_full
echo "tapsum:"; timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "direct:"; FVC_TAPSUM=0 timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],r['achieved'],r['frac_of_x3_ceiling'],r['ms_per_pframe'],d['quality'])"
