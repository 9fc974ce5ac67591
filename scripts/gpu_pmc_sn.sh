#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsn
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SMEM -d gpurun_out/pmcsn/p1 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_128_2_full --iters 2 > gpurun_out/pmcsn/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_LEVEL_LDS -d gpurun_out/pmcsn/p2 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_128_2_full --iters 2 > gpurun_out/pmcsn/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcsn/p3 -o run --output-format csv -- python scripts/conv_micro.py --cases c3_128_2_full --iters 2 > gpurun_out/pmcsn/p3.log 2>&1 || exit 1
python scripts/pmc_summary.py smalln gpurun_out/pmcsn/p1/run_counter_collection.csv gpurun_out/pmcsn/p2/run_counter_collection.csv gpurun_out/pmcsn/p3/run_counter_collection.csv
