#!/bin/bash
# r6: PMC passes over the bench's serial pass, one counter group per rocprofv3 run (each under
# timeout -s KILL); summarised per split-precision family by scripts/pmc_families.py
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
SERIAL="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ref-metrics --serial $EXTRA"
pass() {
  local name=$1; shift
  timeout -s KILL 420 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- $SERIAL \
    --json-out $OUT/bench_$name.json > $OUT/$name.log 2>&1
  local rc=$?; echo "[pmc] $name rc=$rc"; return $rc
}
pass p1 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE || exit 1
pass p2 FETCH_SIZE || exit 1
pass p3 WRITE_SIZE || exit 1
python3 scripts/pmc_families.py $OUT --bench-json $OUT/bench_p1.json --out $OUT/pmc_families.txt
