#!/bin/bash
# x3 kernel iteration: GPU parity suite, conv micro-benchmarks, default bench (no CPU leg)
export TMPDIR=/tmp
O=gpurun_out/${1:-e1}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python scripts/conv_micro.py > $O/conv_micro.log 2>&1 || { tail -20 $O/conv_micro.log; exit 1; }
grep -v amdgpu.ids $O/conv_micro.log
if [ -f fastvideocodec_amd/libfvc_base.so ]; then FVC_LIB_PATH=$PWD/fastvideocodec_amd/libfvc_base.so timeout -k 10 200 python scripts/conv_micro.py > $O/conv_micro_base.log 2>&1 || exit 1; echo base; grep -v amdgpu.ids $O/conv_micro_base.log; fi

timeout -k 10 300 python bench.py --no-cpu-baseline --json-out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'],r['achieved'],r['frac_of_x3_ceiling'],r['ms_per_pframe'],d['quality'])"
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --serial --breakdown > $O/breakdown.log 2>&1 || exit 1
grep -v amdgpu.ids $O/breakdown.log | head -30 | cut -c1-100
