#!/bin/bash
# Compaction offsets by ballots + mbcnt (no shuffle scans): parity, A/B vs the previous build.
set -u
OUT=gpurun_out/r2s36; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '"rep"' $OUT/$name.log | tail -3 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 500 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_signed_zero.py -x -q -k "topk or choco or Choco" --timeout 300 --timeout-method thread
for i in 1 2 3; do
step old$i 200 env MX_GOSSIP_LIB=_ab/lib_prev.so VARIANTS=none REPS=2 python -u tools/choco_mall.py
step new$i 200 env VARIANTS=none REPS=2 python -u tools/choco_mall.py
done
