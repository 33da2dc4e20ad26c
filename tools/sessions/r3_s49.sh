#!/bin/bash
# Round 3, session 49: the wide kernel with two pieces' loads in flight (wide_pf2) -- parity, then
# the slot-count table with it off (default) and on.
set -u
OUT=gpurun_out/r3s49; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py
TAILN=40 WIDE_CASES=72:0.08,96:0.06,128:0.05,150:0.04,156:0.04,48:0.9 WIDE_SWEEP=";wide_pf2=1;wide_pf2=1,wide_lds_kb=80;;wide_pf2=1" step sweep 600 python -u tools/widebench.py
