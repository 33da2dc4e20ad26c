#!/bin/bash
# round 2 session 3: full GPU suite, then the driver's bench command twice, then a kernel variant sweep
set -u
OUT=gpurun_out/r2s3
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -6 $OUT/$name.log | cut -c1-3000; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench1 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0
step gaps 300 python -u tools/gaps.py 100 grid=512 unroll=2 grid=512
