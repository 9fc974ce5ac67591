#!/bin/bash
export TMPDIR=/tmp
for v in "FVC_CONV_X=0" "FVC_CONV_WN2=1" "FVC_CONV_PIPE=1"; do
  echo "== $v"
  env $v timeout -k 10 120 python scripts/conv_micro.py --cases c3_64_full,c3_128_half || exit $?
done > gpurun_out/micro_r1h.log 2>&1
cat gpurun_out/micro_r1h.log
mkdir -p gpurun_out/pmc_r1h
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_r1h -o p1 -- python scripts/conv_micro.py --cases c3_64_full,c7_32_64_full --iters 3 > gpurun_out/pmc_r1h/log1.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_r1h -o p2 -- python scripts/conv_micro.py --cases c3_64_full,c7_32_64_full --iters 3 > gpurun_out/pmc_r1h/log2.txt 2>&1 || exit $?
ls gpurun_out/pmc_r1h
