#!/bin/bash
# Round 3, session 4: rocprofv3 evidence of this tree -- the headline (kernel trace + FETCH / WRITE
# PMC passes), Choco per-kernel traces (one row / 8 rows), and the N > 1 recipe exercised at N = 1.
set -u
OUT=gpurun_out/r3s4; mkdir -p $OUT; export TMPDIR=/tmp
( while true; do date +%T >> $OUT/heartbeat.log; sleep 30; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -14 $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step prof 700 bash tools/profile_round.sh r03a
for G in row1 rows8; do
  CHOCO_GROUP=$G K=30 step choco_$G 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/choco_$G -o choco -- python -u tools/choco_rounds.py
done
step multi1 400 bash tools/profile_multi.sh 1 r03t
