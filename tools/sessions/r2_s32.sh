#!/bin/bash
# compact_blocks sweep (persistent compaction grid over all rows) on the current defaults.
set -u
OUT=gpurun_out/r2s32; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 env REPS=3 VARIANTS="${VARIANTS:-compact_blocks=0,compact_blocks=512,compact_blocks=768,compact_blocks=1280,compact_blocks=1536,compact_blocks=2560,compact_blocks=3072}" python -u tools/choco_mall.py > $OUT/ab.log 2>&1; rc=$?
grep -v '"rep"' $OUT/ab.log | tail -14; exit $rc
