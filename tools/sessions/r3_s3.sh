#!/bin/bash
# Round 3, session 3: config 5's per-GPU shares (er_share: 64 / 63 / 55 / 44 slots, knob
# variants), then the Choco A/B of the folded fallback compaction vs the previous build.
set -u
OUT=gpurun_out/r3s3; mkdir -p $OUT; export TMPDIR=/tmp
( while true; do date +%T >> $OUT/heartbeat.log; sleep 30; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -25 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
ER_P=250000000 VARIANTS="base;ns48=1;blocks_per_cu=1;blocks_per_cu=3;ns48=1,blocks_per_cu=3;nontemporal=0;nontemporal=1" step er_share 500 python -u tools/er_share.py
for i in 1 2 3; do
  VARIANTS=none REPS=1 MX_GOSSIP_LIB=_ab/lib_r03a.so step ab_old_$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=1 step ab_new_$i 200 python -u tools/choco_mall.py
done
