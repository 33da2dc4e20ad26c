#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the bench, then one PMC pass per TCC
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass), each under its own kill limit.
# Headline launches only (--configs 0: the WRN-28-10 figure runs the same kernel instantiation on
# 36.5M-param rows and would skew the per-launch averages).
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --staged 0 --configs 0 --choco 0 --allreduce 0 --er 0"
run() { local lim=$1; shift; echo "== $*"; timeout -k 10 -s KILL $lim "$@"; local rc=$?; echo "rc=$rc"; return $rc; }
run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $BENCH > $OUT/trace.log 2>&1 || exit $?
python tools/gaps.py --trace $(ls $OUT/trace/*kernel_trace.csv $OUT/trace/*/*kernel_trace.csv 2>/dev/null | head -1) > $OUT/mix_gaps.json
PMC_BENCH="python -u bench.py --steps 5 --warmup 2 --cpu-seconds 0 --settle-ms 0 --staged 0 --configs 0 --choco 0 --allreduce 0 --er 0"
run 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $PMC_BENCH > $OUT/fetch.log 2>&1 || exit $?
run 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $PMC_BENCH > $OUT/write.log 2>&1 || exit $?
python tools/pmc_summary.py $OUT $OUT/rocprof_$TAG.json
