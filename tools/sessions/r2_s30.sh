#!/bin/bash
# Final-tree evidence: bench line, rocprofv3 kernel trace + FETCH/WRITE_SIZE passes (profile_round.sh),
# Choco per-kernel traces (one row, 8 rows).
set -u
OUT=gpurun_out/r2s30; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
bash tools/profile_round.sh r02b > $OUT/profile.log 2>&1 || exit $?
for g in row1 rows8; do
  CHOCO_GROUP=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/choco_$g -o choco -- python3 -u tools/choco_rounds.py > $OUT/choco_$g.log 2>&1 || exit $?
done
tail -2 $OUT/profile.log
