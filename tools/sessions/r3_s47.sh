#!/bin/bash
# Round 3, session 47: evidence on the final kernels -- the default bench line, then the rocprof
# kernel-trace + PMC recipe (tools/profile_round.sh r03d).
set -u
OUT=gpurun_out/r3s47; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=1 step bench 600 python -u bench.py
TAILN=6 step prof 900 bash tools/profile_round.sh r03d
