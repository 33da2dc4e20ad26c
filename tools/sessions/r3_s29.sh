#!/bin/bash
# Round 3, session 29: the whole GPU suite (rows_pf2 auto, balanced compaction grid), then the
# driver's default bench command.
set -u
OUT=gpurun_out/r3s29; mkdir -p $OUT; export TMPDIR=/tmp
( while true; do date +%T >> $OUT/heartbeat.log; sleep 30; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-6} $OUT/$name.log | cut -c1-3000; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step suite 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
TAILN=2 step bench 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
