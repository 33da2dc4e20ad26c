#!/bin/bash
set -u
OUT=gpurun_out/r2s9
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -8 $OUT/$name.log | cut -c1-600; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step wide_tests 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread
step wide 300 python -u tools/widebench.py
