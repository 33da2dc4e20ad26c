#!/bin/bash
# Round 3, session 38: wide kernel, LDS budget x workgroups-per-CU sweep (96 / 128 / 150 slots, 48 x 46).
set -u
OUT=gpurun_out/r3s38; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=60 WIDE_CASES=96:0.06,128:0.05,150:0.04,48:0.9 WIDE_SWEEP="wide_lds_kb=40,wide_per_cu=1;wide_lds_kb=40,wide_per_cu=2;wide_lds_kb=40,wide_per_cu=3;wide_lds_kb=40,wide_per_cu=4;wide_lds_kb=80,wide_per_cu=1;wide_lds_kb=80,wide_per_cu=2;wide_lds_kb=80,wide_per_cu=3;wide_lds_kb=80,wide_per_cu=4;wide_lds_kb=158,wide_per_cu=1;wide_lds_kb=158,wide_per_cu=2;wide_lds_kb=158,wide_per_cu=3;wide_lds_kb=158,wide_per_cu=4" step sweep 600 python -u tools/widebench.py
