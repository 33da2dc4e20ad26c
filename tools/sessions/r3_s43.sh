#!/bin/bash
# Round 3, session 43: the wide tests after the LDS-attribute change; config 1 / 2's small rows --
# eager and graph-replayed rounds, and their kernel trace.
set -u
OUT=gpurun_out/r3s43; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step wide 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py -k "wide"
TAILN=6 step small 300 python -u tools/small_cfg.py
TAILN=3 step small_prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o small -- python3 -u tools/small_cfg.py
find $OUT/prof -name "*kernel_stats.csv" | head -3
for f in $(find $OUT/prof -name "*kernel_stats.csv"); do cut -c1-220 $f | head -8; done
