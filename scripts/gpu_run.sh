#!/bin/bash
# One parameterised GPU round trip (replaces the per-experiment launchers of rounds 1-4).
#   bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failing step ends the script.
#   tests            full -m gpu suite, one pytest process
#   tests:EXPR       -m gpu tests selected by -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            default bench (CPU leg + parity block)        -> OUT/bench.json
#   bench-fast       pipelined bench, no CPU leg, STEPS (default 6) -> OUT/bench_fast.json
#   breakdown        serial bench with the per-geometry table on stderr
#   prof             rocprofv3 --kernel-trace --stats of the serial bench
#   pmc              FETCH_SIZE and WRITE_SIZE passes of the serial bench (one counter group a run)
#   micro:ARGS       python scripts/conv_micro.py ARGS
# Environment: EXTRA="--gops-per-gpu 8 ..." is appended to every bench command.
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
STEPS=${STEPS:-6}
SERIAL="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ref-metrics --serial $EXTRA"
run() {  # run NAME SECONDS CMD...: log to OUT/NAME.log, stop the script on failure
  local name=$1 secs=$2; shift 2
  echo "[gpu_run] $name: $*"
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -3 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "[gpu_run] $name failed (exit $rc)"; tail -30 $OUT/$name.log; exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests) run pytest 1100 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread \
             -p no:cacheprovider -rP --tb=short ;;
    tests:*) run pytest_k 900 python -u -m pytest tests -m gpu -v --timeout 420 --timeout-method thread \
             -p no:cacheprovider -rP --tb=short -k "${step#tests:}" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) run bench 900 python -u bench.py --json-out $OUT/bench.json $EXTRA ;;
    bench-fast) run bench_fast 600 python -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --no-ref-metrics \
             --json-out $OUT/bench_fast.json $EXTRA ;;
    breakdown) run breakdown 600 $SERIAL --breakdown ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $SERIAL \
             --json-out $OUT/bench_serial.json ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $SERIAL
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $SERIAL ;;
    micro:*) run micro 600 python -u scripts/conv_micro.py ${step#micro:} ;;
    *) echo "[gpu_run] unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_run] done"
