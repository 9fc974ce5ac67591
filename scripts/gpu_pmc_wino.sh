#!/bin/bash
# PMC passes over one conv geometry on the Winograd kernel (conv_micro, batch 8), one counter group
# per rocprofv3 run under `timeout -s KILL`; then the same for the direct kernel (FVC_WINO=0).
export TMPDIR=/tmp
CASE=${CASE:-c3_64_full}
for V in ${VS:-1 0}; do
OUT=gpurun_out/pmcw${V}_$CASE; mkdir -p $OUT
pass() {
  local name=$1; shift
  FVC_WINO=$V timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
    python scripts/conv_micro.py --cases $CASE --batch 8 --iters 2 > $OUT/$name.log 2>&1
  echo "$V $name rc=$?"
}
pass p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES || exit 1
pass p2 SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA || exit 1
pass p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC || exit 1
for p in p1 p2 p3; do f=$(find $OUT/$p -name "*counter_collection.csv" | head -1); python scripts/pmc_summary.py conv_ $f; done
done
