#!/bin/bash
# probe (not a product build): apply pass with its message phase removed (no partner / own
# entries applied, no dirty granules) vs the real build -- how much of the apply is the message phase.
set -u
OUT=gpurun_out/r2s51; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-4} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
for i in 1 2; do
  MX_GOSSIP_LIB=_ab/lib_probe_nomsg.so VARIANTS=none REPS=2 TAILN=2 step probe$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=2 TAILN=2 step real$i 200 python -u tools/choco_mall.py
done
for g in rows8 row1; do
  MX_GOSSIP_LIB=_ab/lib_probe_nomsg.so CHOCO_GROUP=$g K=30 TAILN=1 step prof_$g 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_$g -o run -- python3 -u tools/choco_rounds.py
done
