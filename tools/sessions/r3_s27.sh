#!/bin/bash
# Round 3, session 27: balanced one-row compaction grid -- parity (top-k patterns, Choco rounds,
# full VGG), then a same-box A/B against the old 640-block grid.
set -u
OUT=gpurun_out/r3s27; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gossip.py tests/test_gpu_configs.py -k "topk or choco or vgg"
TAILN=4 VARIANTS="compact_blocks=640,compact_blocks=0" REPS=4 step ab 300 python -u tools/choco_mall.py
