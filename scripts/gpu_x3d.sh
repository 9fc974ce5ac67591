#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv" > gpurun_out/pytest_x3d.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_x3d.log; [ $rc -eq 0 ] || exit $rc
C=c3_64_full,c3_128_half,c7_32_64_full,d3_128_half,d5_64_quarter,c7_32_16_full
for v in "FVC_X3_WM=2" "FVC_X3_CC=32" "FVC_X3_CC=32 FVC_X3_WN=1"; do
  echo "== $v"; env $v timeout -k 10 120 python scripts/conv_micro.py --cases $C 2>&1 | grep -v amdgpu.ids || exit 1
done
mkdir -p gpurun_out/pmc2
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/pmc2/p1 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_64_full --iters 2 > gpurun_out/pmc2/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA -d gpurun_out/pmc2/p2 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_64_full --iters 2 > gpurun_out/pmc2/p2.log 2>&1 || exit 1
python scripts/pmc_summary.py conv_x3 gpurun_out/pmc2/p1/run_counter_collection.csv gpurun_out/pmc2/p2/run_counter_collection.csv
