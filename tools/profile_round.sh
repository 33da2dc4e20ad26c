#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the bench, then one PMC pass per TCC
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass), each under its own kill limit.
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0"
run() { local lim=$1; shift; echo "== $*"; timeout -k 10 -s KILL $lim "$@"; local rc=$?; echo "rc=$rc"; return $rc; }
run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $BENCH > $OUT/trace.log 2>&1 || exit $?
run 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/fetch.log 2>&1 || exit $?
run 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/write.log 2>&1 || exit $?
python tools/pmc_summary.py $OUT $OUT/rocprof_$TAG.json
