#!/bin/bash
# Round 3, session 9: wave-owned-chunk compaction -- parity (one row / 8 rows, every pattern incl.
# the sampled fallback), then a same-box A/B over chunks per wave.
set -u
OUT=gpurun_out/r3s9; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -16 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step parity 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gossip.py -k "compaction_variants"
VARIANTS="compact_wave=0,compact_wave=1,compact_wave=2,compact_wave=4,compact_wave=8" REPS=3 step mall 300 python -u tools/choco_mall.py
