#!/bin/bash
set -u
OUT=gpurun_out/r2s13; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_pre_nt.so timeout -k 10 120 python -u tools/chocobench.py 2>&1 | grep round_ms | sed 's/^/old /' | cut -c1-120 >> $OUT/ab.log || exit 1
  timeout -k 10 120 python -u tools/chocobench.py 2>&1 | grep round_ms | sed 's/^/new /' | cut -c1-120 >> $OUT/ab.log || exit 1
done
cat $OUT/ab.log
