#!/bin/bash
# Choco knob variants: parity (new knob tests + the Choco/top-k suite), then a same-box A/B of
# compaction stores (masked per element vs looped over kept) and apply granules (64 B vs 32 B).
set -u
OUT=gpurun_out/r2s42; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -12 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py -m gpu -x -q --timeout 200 --timeout-method thread -k "choco or topk"
VARIANTS="compact_store=0:apply_gran=16,compact_store=1,apply_gran=8,compact_store=1:apply_gran=8" REPS=3 step mall 300 python -u tools/choco_mall.py
