#!/bin/bash
# Round 3, session 41: the row kernel's 32-64-slot classes in 512 / 1024-thread workgroups (rows_tpb)
# -- parity, then config 5's per-GPU shares (N = 8 / 4 / 2 / 1) and the slot-count table.
set -u
OUT=gpurun_out/r3s41; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py -k "er64_shares or rows_tpb"
TAILN=30 ER_P=250000000 VARIANTS="base;rows_tpb=512;rows_tpb=1024" step er_share 700 python -u tools/er_share.py
TAILN=30 WIDE_CASES=32:0.15,40:0.12,64:0.1 WIDE_SWEEP="rows_tpb=256;rows_tpb=512;rows_tpb=1024" step sweep 300 python -u tools/widebench.py
