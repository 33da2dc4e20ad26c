#!/bin/bash
# Round 3, session 25: rows_pf2 auto -- parity of the mixing kernels (ER shares, every wide config),
# the share probe with the defaults, and the headline bench (must be unchanged).
set -u
OUT=gpurun_out/r3s25; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_gossip.py tests/test_gpu_configs.py -k "er64 or er_graphs_wide or wide or wrn"
TAILN=6 ER_P=250000000 VARIANTS="base;rows_pf2=0" step er_share 600 python -u tools/er_share.py
TAILN=1 step bench 500 python3 bench.py --gpus 1 --steps 20 --warmup 5
