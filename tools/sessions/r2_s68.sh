#!/bin/bash
# wide kernel (> 64 slots / > 32 matchings): one workgroup per piece vs the persistent grid
# (_ab/lib_widepers.so): wide parity tests, then tools/widebench.py on both builds.
set -u
OUT=gpurun_out/r2s68; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-6} $OUT/$name.log | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 400 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  MX_GOSSIP_LIB=_ab/lib_widepers.so step old$i 300 python -u tools/widebench.py
  step new$i 300 python -u tools/widebench.py
done
