#!/bin/bash
# Round 3, session 6: whole GPU suite + smoke + the driver's default bench command on this tree.
set -u
OUT=gpurun_out/r3s6; mkdir -p $OUT; export TMPDIR=/tmp
( while true; do date +%T >> $OUT/heartbeat.log; sleep 30; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step suite 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
