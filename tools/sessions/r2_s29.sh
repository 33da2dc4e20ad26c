#!/bin/bash
# Apply with compare-found dirty granules (32 KB LDS, 5 blocks/CU): parity, then A/B vs flags.
set -u
OUT=gpurun_out/r2s29; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; grep -v '"rep"' $OUT/$name.log | tail -6 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 500 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_multiproc.py tests/test_gpu_wide.py tests/test_gpu_signed_zero.py tests/test_gpu_harness.py tests/test_gpu_edges.py -x -q -k "choco or Choco" --timeout 300 --timeout-method thread
step ab1 200 env VARIANTS="apply_cmp=0,apply_cmp=1" REPS=3 python -u tools/choco_mall.py
step ab2 200 env VARIANTS="apply_cmp=1,apply_cmp=0" REPS=3 python -u tools/choco_mall.py
