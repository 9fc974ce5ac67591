#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py -m gpu -x -v -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_dbg.log; exit $rc
