#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/k4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -k "4k" -x -q -p no:cacheprovider --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --height 2160 --width 3840 --gop 32 --steps 1 --warmup 1 --no-cpu-baseline --json-out $O/bench_4k.json > $O/bench_4k.log 2>&1 || { tail -20 $O/bench_4k.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_4k.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['achieved'],r['ms_per_pframe'],d['quality'])"
