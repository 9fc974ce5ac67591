#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rans or coder or decode or bitstream or compress" > gpurun_out/pytest_coder.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_coder.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_coder.log; exit $rc; }
timeout -k 10 120 python scripts/coder_micro.py 2>&1 | grep -v amdgpu.ids
