#!/bin/bash
# last tree of round 2 session 4 (auto access hints): whole GPU suite, smoke, default bench
set -u
OUT=gpurun_out/r2s82; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-2} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 400 python -u bench.py
