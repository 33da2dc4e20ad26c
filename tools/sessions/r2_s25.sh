#!/bin/bash
# cand_chunks sweep (fewer candidate-pass blocks = fewer histogram flushes).
set -u
OUT=gpurun_out/r2s25; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 env REPS=3 VARIANTS="cand_chunks=2,cand_chunks=3,cand_chunks=4,cand_chunks=6,cand_chunks=8" python -u tools/choco_mall.py > $OUT/ab.log 2>&1; rc=$?
grep -v '"rep"' $OUT/ab.log | tail -12; exit $rc
