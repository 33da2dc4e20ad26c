#!/bin/bash
# Round 3, session 2: the whole GPU suite (incl. the new multi-process bench / watchdog / deadline
# tests), the default bench, then the ER(64) per-GPU share probe (config 5's 44-slot share).
set -u
OUT=gpurun_out/r3s2; mkdir -p $OUT; export TMPDIR=/tmp
( while true; do date +%T >> $OUT/heartbeat.log; sleep 30; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -15 $OUT/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step suite 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 500 python -u bench.py --steps 20 --warmup 5
ER_P=250000000 VARIANTS="base;ns48=1;blocks_per_cu=1;blocks_per_cu=3;ns48=1,blocks_per_cu=3;nontemporal=0" step er_share 400 python -u tools/er_share.py
# Choco A/B: the fallback compaction folded into the first candidate pass (this tree) vs the r02
# launch sequence (_ab/lib_r03a.so, the previous commit), interleaved
for i in 1 2 3; do
  VARIANTS=none REPS=1 MX_GOSSIP_LIB=_ab/lib_r03a.so step ab_old_$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=1 step ab_new_$i 200 python -u tools/choco_mall.py
done
