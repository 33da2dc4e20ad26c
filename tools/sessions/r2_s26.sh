#!/bin/bash
# Auto cand_chunks (4 / 8), with the write_cand / apply range guards in place: parity, Choco A/B vs HEAD.
set -u
OUT=gpurun_out/r2s26; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '"rep"' $OUT/$name.log | tail -6 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step topk 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_multiproc.py tests/test_gpu_wide.py -x -q -k "topk or choco or Choco" --timeout 200 --timeout-method thread
for i in 1 2; do
step ab_head$i 200 env MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 python -u tools/choco_mall.py
step ab_new$i 200 env VARIANTS="cand_chunks=0,cand_chunks=12" REPS=2 python -u tools/choco_mall.py
done
