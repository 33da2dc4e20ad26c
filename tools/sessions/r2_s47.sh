#!/bin/bash
# compaction grid sweep with the looped-store build (93-95 VGPRs: 5 waves per SIMD).
set -u
OUT=gpurun_out/r2s47; mkdir -p $OUT; export TMPDIR=/tmp
VARIANTS="compact_blocks=2048,compact_blocks=2560,compact_blocks=2888,compact_blocks=3072,compact_blocks=3608,compact_blocks=4096,compact_blocks=640,compact_blocks=768,compact_blocks=896" REPS=3 timeout -k 10 300 python -u tools/choco_mall.py > $OUT/sweep.log 2>&1; rc=$?; tail -12 $OUT/sweep.log; exit $rc
