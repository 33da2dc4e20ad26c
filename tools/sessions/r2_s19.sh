#!/bin/bash
# apply_nt by row count: parity (new top-k patterns too), A/B vs HEAD build.
set -u
OUT=gpurun_out/r2s19; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step topk 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_multiproc.py -x -q -k "topk or choco or Choco" --timeout 200 --timeout-method thread
for i in 1 2; do
step ab_old$i 200 env MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 python -u tools/choco_mall.py
step ab_new$i 200 env VARIANTS=-1,0,1 REPS=2 python -u tools/choco_mall.py
done
