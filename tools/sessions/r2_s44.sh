#!/bin/bash
# looped candidate stores as the default: Choco parity, then per-kernel times (rows8 / row1).
set -u
OUT=gpurun_out/r2s44; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-4} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "choco or topk or vgg"
for g in rows8 row1; do
  CHOCO_GROUP=$g K=30 step prof_$g 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_$g -o run -- python3 -u tools/choco_rounds.py
done
for f in $(find $OUT -name "*kernel_stats.csv"); do echo "## $f"; cut -d, -f1-4 $f | head -9 | cut -c1-150; done
