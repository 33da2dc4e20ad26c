#!/bin/bash
# Final-tree evidence (round 2, session 4, split-2 flat grid):
# (kernel trace + FETCH/WRITE_SIZE passes), Choco kernel traces (8 rows / one row) and Choco PMC
# passes (8 rows) for the compaction / apply byte accounting.
set -u
OUT=gpurun_out/r2s72; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 -s KILL $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-3} $OUT/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step gputests 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step bench 400 python -u bench.py
bash tools/profile_round.sh r02g > $OUT/profile.log 2>&1; rc=$?; tail -3 $OUT/profile.log; [ $rc -eq 0 ] || exit $rc
for g in rows8 row1; do
  CHOCO_GROUP=$g K=30 TAILN=1 step choco_$g 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/choco_$g -o run -- python3 -u tools/choco_rounds.py
done
for c in FETCH_SIZE WRITE_SIZE; do
  CHOCO_GROUP=rows8 K=5 TAILN=1 step choco_pmc_$c 120 rocprofv3 --pmc $c --output-format csv -d $OUT/choco_pmc_$c -o run -- python3 -u tools/choco_rounds.py
done
