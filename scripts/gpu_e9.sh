#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e9; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
C=c3_64_full,c3_128_half,d3_128_half,c7_32_64_full,c3_128_eighth
echo "dyn:"; timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "static:"; FVC_X3_DYN=0 timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('dyn',d['value'],r['achieved'],r['frac_of_x3_ceiling'],r['ms_per_pframe'],d['quality'])"
FVC_X3_DYN=0 timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench_static.json > $O/bench_static.log 2>&1 || { tail -20 $O/bench_static.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_static.json'));r=d['roofline'];print('static',d['value'],r['achieved'],r['frac_of_x3_ceiling'],r['ms_per_pframe'])"
