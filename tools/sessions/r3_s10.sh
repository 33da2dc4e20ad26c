#!/bin/bash
# Round 3, session 10: one-launch selection (select_kernel) -- parity (every pattern, 1 / 5 / 32 / auto
# blocks per row, one row and 8 rows, the sampled fallback), then a same-box A/B against the four passes.
set -u
OUT=gpurun_out/r3s10; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -16 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step parity 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gossip.py -k "select_kernel or work_reuse"
VARIANTS="select=0,select=1,select=1:select_blocks=16,select=1:select_blocks=8" REPS=3 step mall 300 python -u tools/choco_mall.py
