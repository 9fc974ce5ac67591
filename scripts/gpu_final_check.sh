#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/final2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final2/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final2/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final2/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2/smoke.log 2>&1 || { tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
bash scripts/gpu_store_nt.sh
