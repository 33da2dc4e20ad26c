#!/bin/bash
# headline row kernel: next tile's loads issued after the current tile's stores (late) vs right
# after the barrier (early, the default): parity of the late build on the mix tests, bench A/B.
set -u
OUT=gpurun_out/r2s56; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-2} $OUT/$name.log | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
MX_GOSSIP_LIB=_ab/lib_late.so step tests 300 python -u -m pytest tests/test_gpu_gossip.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mix or golden or full"
B="python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --staged 0 --configs 0 --choco 0 --allreduce 0"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_early.so TAILN=1 step early$i 200 $B
  MX_GOSSIP_LIB=_ab/lib_late.so TAILN=1 step late$i 200 $B
done
