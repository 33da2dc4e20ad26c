#!/bin/bash
set -u
OUT=gpurun_out/r2s12
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/choco_nt.py > $OUT/nt.log 2>&1; echo rc=$?; cat $OUT/nt.log | grep case
