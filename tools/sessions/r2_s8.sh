#!/bin/bash
# round 2 session 8: wide-kernel throughput; pull transport overheads with 2 processes on one GPU
set -u
OUT=gpurun_out/r2s8
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -8 $OUT/$name.log | cut -c1-2500; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
step wide 300 python -u tools/widebench.py
step pull2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --transport gloo --steps 10 --warmup 3 --choco 0 --allreduce 0 --cpu-seconds 0
