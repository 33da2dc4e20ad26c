#!/bin/bash
# round 2 session 7: pull transport (multi-process on one GPU), bench exchange forms, full suite
set -u
OUT=gpurun_out/r2s7
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -12 $OUT/$name.log | cut -c1-1500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step mp 900 python -u -m pytest tests/test_gpu_multiproc.py -v -x --timeout 300 --timeout-method thread
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
