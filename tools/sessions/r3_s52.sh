#!/bin/bash
# Round 3, session 52: rocprofv3 kernel trace of the wide-kernel slot table (evidence for the
# widebench rates: per-launch kernel durations of mix_kernel_wide at 96 / 150 slots and 46 matchings).
# (Not run in round 3: the GPU pool had no free box for the last hour of the session; the rates it
# would back are the HIP-event figures in profiles/r03d_wide_kernel_sweep.log / r03d_wide_pf2_ab.log.)
set -u
OUT=gpurun_out/r3s52; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-16} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
TAILN=4 WIDE_CASES=96:0.06,150:0.04,48:0.9 step wide_prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o wide -- python3 -u tools/widebench.py
