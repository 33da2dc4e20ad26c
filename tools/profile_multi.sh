#!/bin/bash
# N > 1 rocprofv3 evidence: the bench under torchrun with EVERY RANK its own
# rocprofv3 process -- torchrun --no-python starts `rocprofv3 ... -- python bench.py` per rank, so
# the profiler's preload starts with the rank's program itself (no launcher process that has touched
# the GPU ever execs another program).  Per-rank kernel traces (the mixing kernel and the RCCL
# kernels, rank-tagged directories), then per-rank PMC passes, each its own run under a kill limit:
#   FETCH_SIZE / WRITE_SIZE    HBM bytes per launch per rank (tools/pmc_summary.py)
#   TCC_EA0_RDREQ_GMI_32B / TCC_EA0_WRREQ_WRITE_GMI_32B   32-byte requests the L2s send over the
#                              fabric to another GPU's memory (reads: the pull transport's partner
#                              rows; writes: RCCL's peer stores), per kernel per rank
# tools/pmc_summary.py --ranks then writes per-rank HBM bytes per launch and xGMI bytes per kernel
# (the mixing kernel's and the RCCL kernels'), for roofline.traffic / xgmi at N > 1.
#
#   bash tools/profile_multi.sh N TAG        (N GPUs of one node; never run it with N > GPUs present)
set -u
N=${1:-8}
TAG=${2:-r03}
OUT=gpurun_out/prof_${TAG}_n${N}
mkdir -p $OUT
export TMPDIR=/tmp
GPUS=$(python -c "import torch; print(torch.cuda.device_count())")
if [ "$GPUS" -lt "$N" ]; then echo "profile_multi: $N ranks need $N GPUs, $GPUS present"; exit 2; fi
PORT=$((20000 + RANDOM % 20000))
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $PORT --no-python"
BENCH="python -u bench.py --gpus $N --steps 20 --warmup 5 --cpu-seconds 0 --staged 0 --configs 0 --choco 0 --allreduce 0 --er 0"
run() { local lim=$1; shift; echo "== $*"; timeout -k 10 -s KILL $lim "$@"; local rc=$?; echo "rc=$rc"; return $rc; }
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run 600 $TR rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace/rank%env{RANK}%" -o "trace_%pid%" -- $BENCH \
    > $OUT/trace.log 2>&1 || exit $?
PMC_BENCH="python -u bench.py --gpus $N --steps 5 --warmup 2 --cpu-seconds 0 --settle-ms 0 --staged 0 --configs 0 --choco 0 --allreduce 0 --er 0"
for C in FETCH_SIZE WRITE_SIZE; do
  run 300 $TR rocprofv3 --pmc $C --output-format csv -d "$OUT/${C,,}/rank%env{RANK}%" -o "pmc_%pid%" -- $PMC_BENCH \
      > $OUT/${C,,}.log 2>&1 || exit $?
done
# xGMI bytes: the L2's fabric requests that leave for another GPU (GMI), in 32-byte units, both
# directions in one pass (2 TCC counters; listed in profiles/r03t_fabric_counters.txt for gfx950)
run 300 $TR rocprofv3 --pmc TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_WRREQ_WRITE_GMI_32B_sum --output-format csv \
    -d "$OUT/fabric_gmi/rank%env{RANK}%" -o "pmc_%pid%" -- $PMC_BENCH > $OUT/fabric_gmi.log 2>&1 || exit $?
python tools/pmc_summary.py --ranks $OUT $OUT/rocprof_${TAG}_n${N}.json
