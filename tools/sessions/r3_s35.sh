#!/bin/bash
# Round 3, session 35: the wide kernel with bigger LDS pieces (wide_lds_kb) -- parity, then the
# slot-count throughput table at 40 (default) / 80 / 158 KB.
set -u
OUT=gpurun_out/r3s35; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=3 step parity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py
for kb in 40 80 158; do TAILN=5 WIDE_TUNE=wide_lds_kb=$kb step wb$kb 300 python -u tools/widebench.py; done
