#!/bin/bash
# round 2 session 2: new parity tests first (config sizes, signed zero, graph checkpoint), then the suite
set -u
OUT=gpurun_out/r2s2
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -15 $OUT/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step new_tests 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_signed_zero.py tests/test_gpu_harness.py -v -x --timeout 300 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
