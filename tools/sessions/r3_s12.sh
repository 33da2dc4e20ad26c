#!/bin/bash
# Round 3, session 12: select_kernel stage clocks (one row, 32 / 16 blocks).
set -u
OUT=gpurun_out/r3s12; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
SEL_B=32 step trace32 120 python -u tools/select_trace.py
SEL_B=16 step trace16 120 python -u tools/select_trace.py
