#!/bin/bash
# PMC passes over one conv_x3_kernel geometry (scripts/conv_micro.py, batch 4): each pass its own
# rocprofv3 run under `timeout -s KILL`, counters limited to the per-pass slots of MI355X_MICROARCH.md
# (8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM); counters the box does not list are dropped.
export TMPDIR=/tmp
CASE=${CASE:-c3_64_full}
OUT=gpurun_out/pmc_$CASE; mkdir -p $OUT
timeout -k 5 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters.txt; }
pass() {
  local name=$1; shift; local list=""
  for c in "$@"; do if have $c; then list="$list $c"; else echo "missing $c" >> $OUT/missing.txt; fi; done
  [ -z "$list" ] && return 0
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $list -d $OUT/$name -o run --output-format csv -- \
    python scripts/conv_micro.py --cases $CASE --batch 4 --iters 2 > $OUT/$name.log 2>&1
  echo "$name rc=$? ($list)"
}
pass p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES || exit 1
pass p2 SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU || exit 1
pass p3 TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_COUNT TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES || exit 1
pass p4 TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_BUSY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CU_CYCLES || exit 1
ls $OUT
