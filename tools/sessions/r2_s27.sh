#!/bin/bash
# Host-model staging in pieces: parity (staging + drop-in tests), bench's staged figure.
set -u
OUT=gpurun_out/r2s27; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_multiproc.py -x -q -k "staging or dropin" --timeout 300 --timeout-method thread
for i in 1 2; do
step bench$i 300 python -u bench.py --steps 5 --warmup 2 --choco 0 --configs 0 --allreduce 0 --cpu-seconds 0
done
