#!/bin/bash
# Round 3, session 26: Choco compaction grid sweep (one row: 3607 chunks -> grids dividing them
# evenly), then the headline rocprofv3 evidence of this tree (kernel trace + FETCH / WRITE PMC).
set -u
OUT=gpurun_out/r3s26; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=16 VARIANTS="compact_blocks=0,compact_blocks=902,compact_blocks=1203,compact_blocks=722,compact_blocks=1804,compact_blocks=3072" REPS=3 step cgrid 400 python -u tools/choco_mall.py
TAILN=4 step prof 700 bash tools/profile_round.sh r03c
