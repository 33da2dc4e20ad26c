#!/bin/bash
# Round 3, session 31: threshold mark + placement fused (mark_write, ticket-ordered look-back) --
# parity of every top-k / Choco test, then a same-box A/B against the two passes.
set -u
OUT=gpurun_out/r3s31; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_wide.py tests/test_gpu_clamps.py -k "topk or choco or vgg or clamp"
TAILN=4 VARIANTS="fuse_mw=0,fuse_mw=1" REPS=4 step ab 300 python -u tools/choco_mall.py
for g in row1 rows8; do
  TAILN=1 TOPK_SET=fuse_mw=1 CHOCO_GROUP=$g step tr_$g 200 rocprofv3 --kernel-trace -d $OUT/tr_$g -o prof -- python3 -u tools/choco_rounds.py
done
python3 tools/trace_db.py $(find $OUT -name "*.db" | sort) | grep -v "at::native\|synth\|rocclr\|plan_kernel\|mt_stream\|draw_kernel"
