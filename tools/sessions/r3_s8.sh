#!/bin/bash
# Round 3, session 8: the selection passes' histograms loaded in one round trip -- top-k / Choco
# parity, then a same-box A/B against the previous build (_ab/lib_r03b.so), interleaved 3x.
set -u
OUT=gpurun_out/r3s8; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step parity 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_clamps.py -k "topk or choco or vgg or clamps"
for i in 1 2 3; do
  VARIANTS=none REPS=1 MX_GOSSIP_LIB=_ab/lib_r03b.so step ab_old_$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=1 step ab_new_$i 200 python -u tools/choco_mall.py
done
