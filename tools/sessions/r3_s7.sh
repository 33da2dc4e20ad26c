#!/bin/bash
# Round 3, session 7: headline mixing-kernel geometry re-sweep on one box (sub-tile split 1 / 2 / 4,
# flat vs persistent grid, access hints), interleaved twice.
set -u
OUT=gpurun_out/r3s7; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; cat $OUT/$name.log | grep variant | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
for i in 1 2; do
  step sweep_$i 200 python -u tools/gaps.py 60 default split=4 split=1 flat_small=0 nontemporal=0 nontemporal=1 blocks_per_cu=3,flat_small=0
done
