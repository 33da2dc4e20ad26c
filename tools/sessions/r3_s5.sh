#!/bin/bash
# Round 3, session 5: parity of the two-chunks-in-flight compaction, then a same-box A/B of it and
# of the compaction grid (one row / 8 rows).
set -u
OUT=gpurun_out/r3s5; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -12 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step parity 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gossip.py -k "two_chunks or sampled_floor or work_reuse or choco"
VARIANTS="compact_pf2=0,compact_pf2=1,compact_blocks=1024,compact_pf2=1:compact_blocks=1024,compact_pf2=1:compact_blocks=384" REPS=3 step mall 300 python -u tools/choco_mall.py
