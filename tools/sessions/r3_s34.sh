#!/bin/bash
# Round 3, session 34: sampled-floor sample size sweep (sample_stride; auto = about 2^18 samples).
set -u
OUT=gpurun_out/r3s34; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=14 VARIANTS="sample_stride=0,sample_stride=28,sample_stride=112,sample_stride=224,sample_stride=448,sample_pieces=2,sample_stride=112:sample_pieces=2" REPS=3 step ab 400 python -u tools/choco_mall.py
