#!/bin/bash
# Same-box A/B on the GPU box: tools/choco_rounds.py (one row and 8 rows) and tools/compact_trace.py
# for each variant, interleaved, 3 times.  A variant is "<library path or empty>|<TOPK_SET knobs>":
#   VARIANTS="abship/lib_old.so| |compact_dyn=1" bash tools/ab_variant.sh <tag>
# (space-separated; the first is another build via MX_GOSSIP_LIB, the others this tree's build with
# mx_topk_set knobs).
set -u
TAG=${1:-ab}
mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=gpurun_out/${TAG}.log
for i in 1 2 3; do
  for V in $VARIANTS; do
    LIBV=${V%%|*}; KN=${V#*|}
    MX_GOSSIP_LIB=$LIBV TOPK_SET=$KN CHOCO_GROUP=row1 K=45 timeout -k 10 120 python -u tools/choco_rounds.py >> $OUT 2>&1 || exit 1
    MX_GOSSIP_LIB=$LIBV TOPK_SET=$KN CHOCO_GROUP=rows8 K=25 timeout -k 10 120 python -u tools/choco_rounds.py >> $OUT 2>&1 || exit 1
    MX_GOSSIP_LIB=$LIBV TOPK_SET=$KN REPS=15 timeout -k 10 120 python -u tools/compact_trace.py >> $OUT 2>&1 || exit 1
  done
done
grep "^{" $OUT
