#!/bin/bash
# row kernel on short rows: one workgroup per work item (flat_small) vs the persistent grid:
# mix / config parity tests, then tools/smallp.py on both builds (same box).
set -u
OUT=gpurun_out/r2s63; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-3} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_configs.py tests/test_gpu_harness.py -m gpu -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  MX_GOSSIP_LIB=_ab/lib_persist.so TAILN=8 step old$i 300 python -u tools/smallp.py 181668 666547 2000000
  TAILN=8 step new$i 300 python -u tools/smallp.py 181668 666547 2000000
done
