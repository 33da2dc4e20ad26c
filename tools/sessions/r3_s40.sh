#!/bin/bash
# Round 3, session 40: wide kernel defaults 1024 threads / 158 KB -- the wide and ER parity files,
# then the slot-count table (incl. 72 / 80 / 156 slots) at the defaults and at the old 256 / 40 KB.
set -u
OUT=gpurun_out/r3s40; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_configs.py -k "wide or er64 or lds or slot"
TAILN=40 WIDE_CASES=64:0.1,72:0.08,80:0.07,96:0.06,128:0.05,150:0.04,156:0.04,48:0.9 WIDE_SWEEP=";wide_tpb=256,wide_lds_kb=40" step sweep 600 python -u tools/widebench.py
