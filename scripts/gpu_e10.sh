#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/e10; mkdir -p $O
C=c3_64_full,c3_64_full_res,c3_128_half,c3_64_half,d3_128_half,c7_32_64_full,c7_32_16_full,c3s2_128_half,c3_128_quarter
echo "NW=8:"; timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
echo "NW=4:"; FVC_X3_NW=4 timeout -k 10 100 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
FVC_X3_NW=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k conv > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
FVC_X3_NW=4 timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench4.json > $O/bench4.log 2>&1 || { tail -20 $O/bench4.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench4.json'));r=d['roofline'];print('NW4',d['value'],r['achieved'],r['frac_of_x3_ceiling'],r['ms_per_pframe'],d['quality']['decoder_bitexact'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench8.json > $O/bench8.log 2>&1 || { tail -20 $O/bench8.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench8.json'));r=d['roofline'];print('NW8',d['value'],r['achieved'],r['frac_of_x3_ceiling'],r['ms_per_pframe'])"
