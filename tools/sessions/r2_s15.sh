#!/bin/bash
# Choco access-variant A/B (Infinity Cache reuse between the top-k and apply passes).
set -u
OUT=gpurun_out/r2s15; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/choco_mall.py > $OUT/mall.log 2>&1; rc=$?
tail -12 $OUT/mall.log; exit $rc
