#!/bin/bash
# Top-k v2 (small window, LDS-aggregated edge list, select folded into write_cand): parity, A/B, profile.
set -u
OUT=gpurun_out/r2s18; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step topk 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -x -q -k "topk or choco or Choco" --timeout 200 --timeout-method thread
step ab_old 200 env MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 python -u tools/choco_mall.py
step ab_new 200 env VARIANTS=110,000 REPS=2 python -u tools/choco_mall.py
step ab_old2 200 env MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 python -u tools/choco_mall.py
step ab_new2 200 env VARIANTS=110,000 REPS=2 python -u tools/choco_mall.py
for g in row1 rows8; do
  D=$OUT/prof_$g
  CHOCO_GROUP=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D -o prof -- python3 -u tools/choco_rounds.py > $D.log 2>&1 || exit 1
done
