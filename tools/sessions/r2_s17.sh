#!/bin/bash
# Per-kernel Choco times, old (HEAD) vs new top-k, one row and 8 rows.
set -u
OUT=gpurun_out/r2s17; mkdir -p $OUT; export TMPDIR=/tmp
NEW=$PWD/270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd/_native/libmatcha_gossip.so
for g in row1 rows8; do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/_ab/lib_head.so; else L=$NEW; fi
    D=$OUT/${g}_${v}
    MX_GOSSIP_LIB=$L CHOCO_GROUP=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D -o prof -- python3 -u tools/choco_rounds.py > $D.log 2>&1 || exit 1
    for f in $(find $D -name "*kernel_stats.csv"); do python3 tools/kstats.py $f > $D.stats.txt; done
    echo "== $g $v"; cut -c1-40,83- $D.stats.txt | head -12
  done
done
