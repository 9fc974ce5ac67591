#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc1/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|TCP_[A-Z0-9_]*\|TCC_[A-Z0-9_]*\|TA_[A-Z0-9_]*\|GRBM_[A-Z0-9_]*\|FETCH_SIZE\|WRITE_SIZE" gpurun_out/pmc1/counters.txt | sort -u > gpurun_out/pmc1/names.txt
wc -l gpurun_out/pmc1/names.txt
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/pmc1/p1 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_64_full --iters 2 > gpurun_out/pmc1/p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_SMEM -d gpurun_out/pmc1/p2 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_64_full --iters 2 > gpurun_out/pmc1/p2.log 2>&1; echo "p2 rc=$?"
find gpurun_out/pmc1 -name "*counter_collection.csv"
