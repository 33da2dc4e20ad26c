#!/bin/bash
# Round 3, session 13: select_kernel with batched LDS reads and a one-scan write stage.
set -u
OUT=gpurun_out/r3s13; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gossip.py -k "select_kernel or work_reuse"
TAILN=9 SEL_B=29 step trace29 120 python -u tools/select_trace.py
TAILN=9 VARIANTS="select=0,select=1,select=1:select_blocks=32" REPS=3 step mall 300 python -u tools/choco_mall.py
