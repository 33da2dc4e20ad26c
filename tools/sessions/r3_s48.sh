#!/bin/bash
# Round 3, session 48: the extended grid / wide-kernel parity cases.
set -u
OUT=gpurun_out/r3s48; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gossip.py tests/test_gpu_wide.py -k "persistent_and_flat or lds_budget"
