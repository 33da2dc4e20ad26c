#!/bin/bash
# one-row compaction with ordinary (cacheable) loads vs streaming loads (_ab/lib_cnt.so): Choco
# parity, then same-box A/B.
set -u
OUT=gpurun_out/r2s83; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-2} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py -m gpu -x -q --timeout 200 --timeout-method thread -k "choco or topk"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_cnt.so VARIANTS=none REPS=2 step old$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=2 step new$i 200 python -u tools/choco_mall.py
done
