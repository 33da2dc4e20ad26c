#!/bin/bash
# bench with the Choco roofline / one-row share fields; bench-driven tests.
set -u
OUT=gpurun_out/r2s20; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_tests 400 python -u -m pytest tests/test_gpu_multiproc.py -x -q -k "single_gpu or bench" --timeout 300 --timeout-method thread
