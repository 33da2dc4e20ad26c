#!/bin/bash
# Guards in write_cand / apply: parity; then the cost of one extra histogram flush (to a dummy
# array, results unchanged) in the compaction and in cand_hist<10>.
set -u
OUT=gpurun_out/r2s24; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step topk 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -x -q -k "topk or choco or Choco" --timeout 200 --timeout-method thread
NEW=$PWD/270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd/_native/libmatcha_gossip.so
for g in row1 rows8; do
  for v in cur df2 df4; do
    if [ $v = cur ]; then L=$NEW; else L=$PWD/_ab/lib_$v.so; fi
    D=$OUT/${g}_${v}
    MX_GOSSIP_LIB=$L CHOCO_GROUP=$g timeout -k 10 120 rocprofv3 --kernel-trace -d $D -o prof -- python3 -u tools/choco_rounds.py > $D.log 2>&1 || exit 1
  done
done
