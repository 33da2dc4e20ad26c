#!/bin/bash
# (1) headline row kernel: full-tile path with static load / store counts (waits for the next tile's
#     loads only): GPU suite, then same-box A/B of bench.py (headline only) against _ab/lib_nofast.so;
# (2) compaction with whole / partial chunks in separate loops: Choco A/B against _ab/lib_head2.so.
set -u
OUT=gpurun_out/r2s55; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-2} $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
B="python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --staged 0 --configs 0 --choco 0 --allreduce 0"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_nofast.so TAILN=1 step bench_old$i 200 $B
  TAILN=1 step bench_new$i 200 $B
done
for i in 1 2; do
  MX_GOSSIP_LIB=_ab/lib_head2.so VARIANTS=none REPS=2 step choco_old$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=2 step choco_new$i 200 python -u tools/choco_mall.py
done
