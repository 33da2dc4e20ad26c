#!/bin/bash
# Re-submit a gpurun call only while gpurun itself reports "no box / transient" (rc 3: nothing ran,
# nothing charged).  Any other outcome -- including a failing or faulting command -- is final.
OUTF=$1; shift
for attempt in 1 2 3 4 5 6; do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > "$OUTF" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then exit $rc; fi
  grep -q "status=transient\|backing off\|no box" "$OUTF" || exit $rc
  sleep $((attempt * 40))
done
exit 3
