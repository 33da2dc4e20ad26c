#!/bin/bash
# HBM stream probes: copy / read / write rates and the Choco compaction's read pattern piece by piece.
set -u
OUT=gpurun_out/r2s41; mkdir -p $OUT; export TMPDIR=/tmp
PROBE_ROWS=1 timeout -k 10 240 ./tools/hbm_probe > $OUT/probe.log 2>&1; rc=$?; tail -40 $OUT/probe.log; exit $rc
