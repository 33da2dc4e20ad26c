#!/bin/bash
# rocprofv3 kernel-trace stats of the Choco apply forms and the pull fetch kernel
# (tools/choco_slots_ab.py: strided / slot table / persistent applies at 8 / 4 / 2 / 1 rows of the
# VGG-16 size, mx_pull_fetch of the received slots), one process, for profiles/.
set -u
TAG=${1:-r05}
OUT=gpurun_out/prof_choco_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python -u tools/choco_slots_ab.py > $OUT/ab.log 2>&1
