#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault / abort / timeout (rc >= 124 or signal) ends the
# script, an ordinary test failure (rc 1) does not stop the bench.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name" ; date +%T
  timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "rc=$rc"; tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 400 python -u bench.py --steps 50 --warmup 10
  cp $OUT/bench.log $OUT/bench.json
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0
fi
