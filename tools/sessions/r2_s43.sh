#!/bin/bash
# compaction with one load point for whole and partial chunks (no mid-iteration vmcnt(0)):
# parity, then same-box A/B against the HEAD build (_ab/lib_head.so).
set -u
OUT=gpurun_out/r2s43; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-6} $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "choco or topk or vgg"
for i in 1 2; do
  MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 TAILN=2 step head$i 200 python -u tools/choco_mall.py
  VARIANTS="compact_store=0,compact_store=1" REPS=2 TAILN=4 step new$i 200 python -u tools/choco_mall.py
done
