#!/bin/bash
# Full -m gpu suite + smoke on the current tree.
set -u
OUT=gpurun_out/r2s22; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
