#!/bin/bash
# Round-4 GPU pass: the configs[3] 4K GOP-32 test, then the rest of the suite, the default bench
# line and the configs[3] per-rank bench line.
export TMPDIR=/tmp
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -s --timeout 420 --timeout-method thread -k 4k_gop32 > $OUT/pytest_4k.log 2>&1 || { tail -40 $OUT/pytest_4k.log; exit 1; }
grep "4K frame" $OUT/pytest_4k.log; tail -1 $OUT/pytest_4k.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread --deselect tests/test_gpu_configs.py::test_4k_gop32_one_rank_share > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 420 python -u bench.py --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || { tail -30 $OUT/bench_default.log; exit 1; }
tail -c 600 $OUT/bench_default.json
timeout -k 10 420 python -u bench.py --height 2160 --width 3840 --gop 32 --gops-per-gpu 1 --steps 2 --warmup 1 \
  --cpu-baseline quick --json-out $OUT/bench_4k_gop32_1gpu.json > $OUT/bench_4k.log 2>&1 || { tail -30 $OUT/bench_4k.log; exit 1; }
tail -c 300 $OUT/bench_4k_gop32_1gpu.json
