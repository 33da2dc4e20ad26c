# Same-box A/B of mx_topk_set knob values on the Choco round (tools/choco_rounds.py), interleaved:
#   KNOB=apply_pf VALUES="1 2" REPS=3 bash tools/choco_ab.sh
set -u
for rep in $(seq 1 ${REPS:-3}); do
  for grp in rows8 row1; do
    for v in ${VALUES}; do
      echo -n "$grp $KNOB=$v rep=$rep "
      CHOCO_GROUP=$grp K=${K:-40} TOPK_SET=$KNOB=$v timeout -k 10 120 python tools/choco_rounds.py 2>/dev/null | tail -1 || exit 1
    done
  done
done
