#!/bin/bash
# Round 3, session 11: select_kernel with every slot load in flight -- quick parity, A/B, kernel traces.
set -u
OUT=gpurun_out/r3s11; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step parity 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gossip.py -k "select_kernel and (2000001 or layers)"
TAILN=8 VARIANTS="select=0,select=1,select=1:select_blocks=16,select=1:select_blocks=24" REPS=3 step mall 300 python -u tools/choco_mall.py
for v in "row1 select=1" "rows8 select=1" "rows8 select=1:select_blocks=16"; do
  set -- $v; g=$1; ks=$2; tag=${g}_$(echo $ks | tr ':=' '__')
  TAILN=2 CHOCO_GROUP=$g TOPK_SET=$ks step tr_$tag 200 rocprofv3 --kernel-trace --stats -d $OUT/tr_$tag -o prof -- python3 -u tools/choco_rounds.py
done
find $OUT -name "*kernel_stats.csv" | while read f; do echo "## $f"; cut -d, -f1-4 $f | head -10 | cut -c1-160; done
