#!/bin/bash
set -u
OUT=gpurun_out/r2s28; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/staging_ab.py > $OUT/ab.log 2>&1; rc=$?; tail -2 $OUT/ab.log; exit $rc
