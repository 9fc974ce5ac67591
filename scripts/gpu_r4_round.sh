#!/bin/bash
# Round-4 milestone on the GPU: the whole -m gpu suite, smoke(), the default bench line, then the
# profile set (rocprofv3 kernel-trace + stats of the serial bench, FETCH_SIZE and WRITE_SIZE passes).
export TMPDIR=/tmp
OUT=gpurun_out/r4m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 420 python -u bench.py --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || { tail -30 $OUT/bench_default.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print('value', d['value'], 'x3frac', d['roofline']['frac_of_x3_ceiling'])"
bash scripts/gpu_profile_round.sh r4 > $OUT/profile.log 2>&1 || { tail -20 $OUT/profile.log; exit 1; }
tail -3 $OUT/profile.log
