#!/bin/bash
# Round 3, session 39: wide kernel with 512 / 1024-thread workgroups -- parity, then the
# workgroup-size x LDS-budget sweep.
set -u
OUT=gpurun_out/r3s39; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py
TAILN=60 WIDE_CASES=96:0.06,128:0.05,150:0.04,48:0.9 WIDE_SWEEP="wide_tpb=256,wide_lds_kb=40;wide_tpb=256,wide_lds_kb=80;wide_tpb=256,wide_lds_kb=158;wide_tpb=512,wide_lds_kb=40;wide_tpb=512,wide_lds_kb=80;wide_tpb=512,wide_lds_kb=158;wide_tpb=1024,wide_lds_kb=40;wide_tpb=1024,wide_lds_kb=80;wide_tpb=1024,wide_lds_kb=158" step sweep 600 python -u tools/widebench.py
