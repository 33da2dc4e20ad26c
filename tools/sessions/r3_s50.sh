#!/bin/bash
# Round 3, session 50: final tree -- the whole GPU suite, smoke, and the default bench line.
set -u
OUT=gpurun_out/r3s50; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=4 step suite 1050 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
TAILN=2 step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step bench 600 python -u bench.py
