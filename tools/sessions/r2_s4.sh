#!/bin/bash
# round 2 session 4: multiprocess + bench tests (centralized reference order, self-checks), ramp probe
set -u
OUT=gpurun_out/r2s4
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -8 $OUT/$name.log | cut -c1-3000; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step mp_tests 900 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_edges.py tests/test_gpu_harness.py -v -x --timeout 300 --timeout-method thread
step ramp 200 python -u tools/ramp.py
