#!/bin/bash
# Round 3, session 1: the new GPU tests (apply clamps, mean_rows > 64 rows, RCCL deadline), the
# multi-process bench paths (every figure self-checked by the oracle, watchdog), then the default
# bench (incl. the ER(64) 1e9 sweep).  A heartbeat file shows progress of long single tests.
set -u
OUT=gpurun_out/r3s1; mkdir -p $OUT; export TMPDIR=/tmp
( while true; do date +%T >> $OUT/heartbeat.log; sleep 30; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -15 $OUT/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step new 300 $PYT tests/test_gpu_clamps.py tests/test_gpu_edges.py -k "clamps or mean_rows"
step multiproc 900 $PYT tests/test_gpu_multiproc.py
step bench 500 python -u bench.py --steps 20 --warmup 5
