#!/bin/bash
# CU-reserve sweep of the pipelined bench at the 4-GOP default (the reserve leaves CUs of the
# persistent conv grids to the rANS / decode side streams). RESERVES overrides the list; extra
# "name:VAR=V" arguments run the bench once more per spec at the first reserve (A/B of options).
export TMPDIR=/tmp
O=gpurun_out/reserve
mkdir -p $O
RESERVES=${RESERVES:-"40 16 24 32 48 64"}
run() {  # name reserve env...
  local name=$1 r=$2; shift 2
  env FVC_PIPELINE_CU_RESERVE=$r "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$name.log 2>&1 \
    || { tail -20 $O/bench_$name.log; exit 1; }
  echo "$name (reserve $r $*): $(tail -1 $O/bench_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in $RESERVES; do run r$r $r; done
first=${RESERVES%% *}
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}; vars=${vars//,/ }
  run $name $first $vars
done
