#!/bin/bash
# Round 3, session 32: mark_write chunks per block sweep vs the two passes.
set -u
OUT=gpurun_out/r3s32; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gossip.py -k "knob_variants or work_reuse"
TAILN=12 VARIANTS="fuse_mw=0,fuse_mw=1:mw_chunks=4,fuse_mw=1:mw_chunks=8,fuse_mw=1:mw_chunks=12,fuse_mw=1:mw_chunks=16,fuse_mw=1:mw_chunks=32" REPS=3 step ab 400 python -u tools/choco_mall.py
