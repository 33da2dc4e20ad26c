#!/bin/bash
# Round 3, session 22: row-group pipelining of the top-k over two streams (pipe_groups) -- parity,
# then a same-box A/B of group counts and per-group compaction grids (8 rows).
set -u
OUT=gpurun_out/r3s22; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gossip.py -k "knob_variants or work_reuse"
TAILN=12 VARIANTS="pipe_groups=1,pipe_groups=2,pipe_groups=4,pipe_groups=8,pipe_groups=2:pipe_blocks=768,pipe_groups=4:pipe_blocks=512,pipe_groups=2:pipe_blocks=1280" REPS=3 step mall 400 python -u tools/choco_mall.py
