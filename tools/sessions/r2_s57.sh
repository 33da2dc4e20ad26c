#!/bin/bash
# knob re-sweep on the final Choco kernels: candidate-pass chunks per wave, compaction grid
set -u
OUT=gpurun_out/r2s57; mkdir -p $OUT; export TMPDIR=/tmp
VARIANTS="cand_chunks=0,cand_chunks=2,cand_chunks=4,cand_chunks=8,cand_chunks=16,compact_blocks=512,compact_blocks=768,compact_blocks=2048,compact_blocks=3072" REPS=3 timeout -k 10 400 python -u tools/choco_mall.py > $OUT/sweep.log 2>&1; rc=$?; grep round_us_min $OUT/sweep.log; exit $rc
