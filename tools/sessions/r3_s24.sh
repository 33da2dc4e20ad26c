#!/bin/bash
# Round 3, session 24: two tiles' loads in flight in the persistent row kernel (rows_pf2) for
# config 5's per-GPU shares -- parity, then the share probe.
set -u
OUT=gpurun_out/r3s24; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_gossip.py -k "er64_shares or er_graphs_wide"
TAILN=30 ER_P=250000000 VARIANTS="base;rows_pf2=1;ns48=1;ns48=1,rows_pf2=1" step er_share 600 python -u tools/er_share.py
