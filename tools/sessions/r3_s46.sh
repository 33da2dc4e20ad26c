#!/bin/bash
# Round 3, session 46: 8-slot mid-sized rows on a persistent grid of 4 workgroups per CU (mid_bpc) --
# the mixing parity files, then the size sweep with the mode on (default) and off.
set -u
OUT=gpurun_out/r3s46; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_gossip.py -k "not vgg and not er64_config"
TAILN=40 SMALL_P=181668,400000,666547,1000000,2000000,3000000,4000000 SMALL_TUNE=";mid_bpc=0;mid_tiles=12;mid_tiles=16" step sweep 600 python -u tools/small_cfg.py
