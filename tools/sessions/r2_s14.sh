#!/bin/bash
# Re-entry check: full -m gpu suite, smoke, default bench on the restored tree.
set -u
OUT=gpurun_out/r2s14
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -5 $OUT/$name.log | cut -c1-800; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
