#!/bin/bash
# Round 3, session 17: select_kernel with uniform values in SGPRs (no spill, no store wait in the
# placement loop) -- parity, stage clocks, same-box A/B against the HEAD build.
set -u
OUT=gpurun_out/r3s17; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gossip.py -k "select_kernel or work_reuse or knob_variants"
TAILN=9 SEL_B=29 step trace29 120 python -u tools/select_trace.py
for r in 1 2; do
  TAILN=4 MX_GOSSIP_LIB=_ab/lib_head.so VARIANTS=none REPS=2 step head$r 200 python -u tools/choco_mall.py
  TAILN=4 VARIANTS="select=0,select=1" REPS=2 step new$r 200 python -u tools/choco_mall.py
done
