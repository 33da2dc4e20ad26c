#!/bin/bash
# apply with two blocks per 4096-element chunk (apply_parts 2: half the LDS, more blocks per CU):
# Choco parity (incl. the knob variants and message shapes), then a same-box knob A/B.
set -u
OUT=gpurun_out/r2s77; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-6} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "choco or topk or vgg or apply"
VARIANTS="apply_parts=1,apply_parts=2" REPS=4 step mall 300 python -u tools/choco_mall.py
