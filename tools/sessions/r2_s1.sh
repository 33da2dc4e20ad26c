#!/bin/bash
# round 2 session 1: GPU tests, inter-launch gap of the headline round (plain + kernel trace)
set -u
OUT=gpurun_out/r2s1
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -4 $OUT/$name.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step gaps 300 python -u tools/gaps.py 100 default grid=500 grid=1000 blocks_per_cu=3 grid=512
step gaps_trace 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python -u tools/gaps.py 100 default
python tools/gaps.py --trace $(ls $OUT/tr/*/*kernel_trace.csv $OUT/tr/*kernel_trace.csv 2>/dev/null | head -1) > $OUT/gaps_trace_summary.log 2>&1; cat $OUT/gaps_trace_summary.log
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
