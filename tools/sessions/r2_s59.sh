#!/bin/bash
# fused 10+9-bit candidate pass (h19): Choco parity + same-box A/B against the two-pass build:
# same-box A/B against the build before (_ab/lib_nofuse.so), per-kernel times.
set -u
OUT=gpurun_out/r2s59; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-4} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "choco or topk or vgg or apply"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_nofuse.so VARIANTS=none REPS=2 TAILN=2 step old$i 200 python -u tools/choco_mall.py
  VARIANTS=none REPS=2 TAILN=2 step new$i 200 python -u tools/choco_mall.py
done
for g in rows8 row1; do
  CHOCO_GROUP=$g K=30 TAILN=1 step prof_$g 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_$g -o run -- python3 -u tools/choco_rounds.py
done
