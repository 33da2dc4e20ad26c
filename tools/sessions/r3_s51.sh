#!/bin/bash
# Round 3, session 51: Choco candidate-pass grid (cand_chunks) and 8-row compaction grid sweeps.
set -u
OUT=gpurun_out/r3s51; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=10 REPS=3 VARIANTS="cand_chunks=0,cand_chunks=2,cand_chunks=4,cand_chunks=8,cand_chunks=16" step chunks 600 python -u tools/choco_mall.py
TAILN=10 REPS=3 VARIANTS="compact_blocks=0,compact_blocks=1536,compact_blocks=2048,compact_blocks=3072,compact_blocks=4096" step cblocks 600 python -u tools/choco_mall.py
