#!/bin/bash
# Compaction register budget (5 waves/SIMD, 96 VGPRs) x persistent grid sizes.
set -u
OUT=gpurun_out/r2s21; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '"rep"' $OUT/$name.log | tail -12 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step topk 300 python -u -m pytest tests/test_gpu_gossip.py -x -q -k "topk_sampled_floor" --timeout 200 --timeout-method thread
step ab 300 env REPS=3 VARIANTS="compact_occ=4,compact_occ=5,compact_occ=5:compact_blocks=1280,compact_occ=5:compact_blocks=2560,compact_occ=4:compact_blocks=1024,compact_occ=5:compact_blocks=1024" python -u tools/choco_mall.py
