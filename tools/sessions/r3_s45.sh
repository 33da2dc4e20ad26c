#!/bin/bash
# Round 3, session 45: 8-slot rows of 0.18-8M params -- flat grid (one workgroup per work item,
# default) vs the persistent grid at 2 / 4 / 8 workgroups per CU.
set -u
OUT=gpurun_out/r3s45; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=40 SMALL_P=181668,400000,666547,1000000,2000000,4000000,8000000 SMALL_TUNE=";flat_small=0;flat_small=0,blocks_per_cu=4;flat_small=0,blocks_per_cu=8;flat_small=0,blocks_per_cu=3" step sweep 600 python -u tools/small_cfg.py
