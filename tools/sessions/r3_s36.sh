#!/bin/bash
# Round 3, session 36: the wide kernel with its plan record in LDS and four row chains per wave --
# parity, then the slot-count throughput table (plan in LDS at 40 / 80 KB pieces; global plan at 40).
set -u
OUT=gpurun_out/r3s36; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py
TAILN=5 step wb40 300 python -u tools/widebench.py
TAILN=5 WIDE_TUNE=wide_plan_lds=0 step wb40g 300 python -u tools/widebench.py
TAILN=5 WIDE_TUNE=wide_lds_kb=80 step wb80 300 python -u tools/widebench.py
