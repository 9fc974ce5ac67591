#!/bin/bash
# r4: Winograd finishing-mapping A/B, then the coder / forward / GOP tests on the segment framing,
# then a short bench line with the batch-1 reference-comparable figures.
export TMPDIR=/tmp
OUT=gpurun_out/r4c; mkdir -p $OUT
TAG=r4c/wv VARS="pkpf fm" bash scripts/gpu_wino_variants.sh > $OUT/wv.txt 2>&1 || { tail -30 $OUT/wv.txt; exit 1; }
grep -v amdgpu $OUT/wv.txt | tail -30
timeout -k 10 900 python -u -m pytest tests/test_gpu_coder.py tests/test_gpu_forward.py tests/test_gpu_tree_gop.py -m gpu -x -q \
  --timeout 420 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --cpu-baseline none --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], json.dumps(d['reference_comparable'])[:900])"
