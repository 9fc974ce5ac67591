#!/bin/bash
# PMC passes (one run each) on the 3x3 64->64 1080p conv: issue/wait breakdown, LDS, memory
export TMPDIR=/tmp
O=gpurun_out/pmc4
mkdir -p $O
C="python scripts/conv_micro.py --cases c3_64_full --iters 2"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $O/p1 -o run --output-format csv -- $C > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA -d $O/p2 -o run --output-format csv -- $C > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_ADDR_CONFLICT -d $O/p3 -o run --output-format csv -- $C > $O/p3.log 2>&1 || { tail -5 $O/p3.log; echo p3 failed; }
FVC_X3_BLDS=0 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $O/p4 -o run --output-format csv -- $C > $O/p4.log 2>&1 || exit 1
for p in p1 p2 p3 p4; do F=$(find $O/$p -name "*counter_collection.csv" | head -1); [ -n "$F" ] && python scripts/pmc_summary.py conv_x3 $F; done

