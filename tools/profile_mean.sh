#!/bin/bash
# rocprofv3 evidence for the centralized mean (mx_mean_rows_to over 8 x 25.6M in place,
# tools/mean_ab.py): kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in passes of their own.
set -u
TAG=${1:-r04}
OUT=gpurun_out/prof_mean_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() { local lim=$1; shift; echo "== $*"; timeout -k 10 -s KILL $lim "$@"; local rc=$?; echo "rc=$rc"; return $rc; }
run 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python tools/mean_ab.py > $OUT/trace.log 2>&1 || exit $?
run 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python tools/mean_ab.py > $OUT/fetch.log 2>&1 || exit $?
run 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python tools/mean_ab.py > $OUT/write.log 2>&1 || exit $?
python tools/pmc_summary.py $OUT $OUT/rocprof_mean_$TAG.json
