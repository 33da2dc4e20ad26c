#!/bin/bash
# round 2 session 5: wide-layout tests, full suite, driver bench, rocprof evidence
set -u
OUT=gpurun_out/r2s5
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 $OUT/$name.log | cut -c1-1500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step wide 400 python -u -m pytest tests/test_gpu_wide.py -v -x --timeout 200 --timeout-method thread
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
bash tools/profile_round.sh r02 > $OUT/profile.log 2>&1; echo "profile rc=$?"; tail -5 $OUT/profile.log
