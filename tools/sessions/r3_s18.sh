#!/bin/bash
# Round 3, session 18: per-kernel traces, HEAD build vs this build (select 0 / 1), one row and 8 rows.
set -u
OUT=gpurun_out/r3s18; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi; return 0; }
for g in row1 rows8; do
  MX_GOSSIP_LIB=_ab/lib_head.so CHOCO_GROUP=$g step head_$g 200 rocprofv3 --kernel-trace -d $OUT/head_$g -o prof -- python3 -u tools/choco_rounds.py
  TOPK_SET=select=0 CHOCO_GROUP=$g step new0_$g 200 rocprofv3 --kernel-trace -d $OUT/new0_$g -o prof -- python3 -u tools/choco_rounds.py
  TOPK_SET=select=1 CHOCO_GROUP=$g step new1_$g 200 rocprofv3 --kernel-trace -d $OUT/new1_$g -o prof -- python3 -u tools/choco_rounds.py
done
python3 tools/trace_db.py $(find $OUT -name "*.db" | sort) > $OUT/summary.txt; cat $OUT/summary.txt | grep -v "at::native\|synth\|rocclr\|plan_kernel\|mt_stream\|draw_kernel"
