#!/bin/bash
set -u
OUT=gpurun_out/r2s11
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
MX_TOPK_STREAMS=2 step tests 300 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -x -q -k "choco" --timeout 200 --timeout-method thread
for i in 1 2 3; do
  for S in 1 2 4; do MX_TOPK_STREAMS=$S timeout -k 10 120 python -u tools/chocobench.py | sed "s/^/S=$S /" >> $OUT/ab.log 2>&1 || exit 1; done
done
grep round_ms $OUT/ab.log | cut -c1-140
