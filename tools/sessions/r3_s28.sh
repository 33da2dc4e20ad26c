#!/bin/bash
# Round 3, session 28: two chunks in flight in the compaction (compact_pf2) on the chunk-balanced
# one-row grids.
set -u
OUT=gpurun_out/r3s28; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=16 VARIANTS="compact_pf2=0,compact_pf2=1,compact_pf2=1:compact_blocks=602,compact_pf2=1:compact_blocks=516,compact_pf2=1:compact_blocks=902,compact_pf2=0:compact_blocks=602" REPS=3 step pf2 400 python -u tools/choco_mall.py
