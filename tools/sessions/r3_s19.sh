#!/bin/bash
# Round 3, session 19: where the four-pass path lost time -- HEAD vs this build without the select
# slots (layout as HEAD) vs this build, same box, interleaved.
set -u
OUT=gpurun_out/r3s19; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
for r in 1 2; do
  TAILN=2 MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 step head$r 200 python -u tools/choco_mall.py
  TAILN=2 MX_GOSSIP_LIB=_ab/lib_nopub.so VARIANTS=select=0 REPS=2 step nopub$r 200 python -u tools/choco_mall.py
  TAILN=4 VARIANTS="select=0,select=1" REPS=2 step new$r 200 python -u tools/choco_mall.py
done
