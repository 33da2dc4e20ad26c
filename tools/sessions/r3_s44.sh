#!/bin/bash
# Round 3, session 44: configs 1 / 2 small rows -- sub-tile split / flat-grid / non-temporal sweep.
set -u
OUT=gpurun_out/r3s44; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=40 SMALL_TUNE=";split=1;split=2;split=4;flat_small=0;flat_small=0,blocks_per_cu=4;nontemporal=0;nontemporal=1;unroll=2;unroll=4" step sweep 600 python -u tools/small_cfg.py
