#!/bin/bash
# configs[4] view mode on one GPU (8 views -> all on rank 0) and the default line under torchrun.
export TMPDIR=/tmp
O=gpurun_out/views
mkdir -p $O
timeout -k 10 300 python bench.py --views 8 --no-cpu-baseline --json-out $O/bench_views8_1gpu.json > $O/views8.log 2>&1 \
  || { tail -20 $O/views8.log; exit 1; }
tail -1 $O/views8.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --no-cpu-baseline > $O/torchrun1.log 2>&1 || { tail -20 $O/torchrun1.log; exit 1; }
tail -1 $O/torchrun1.log | cut -c1-300
