#!/bin/bash
# Round 3, session 30: headline kernel A/B, the build before the row-kernel prefetch change
# (_ab/lib_head.so = f49b26c) vs this tree, interleaved on one box (headline figure only).
set -u
OUT=gpurun_out/r3s30; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi; python3 -c "
import json,sys
l=[x for x in open('$OUT/$name.log') if x.startswith('{\"metric')][0]; d=json.loads(l); r=d['roofline']
print('$name', round(d['ms_per_step'],5), round(r['avg_launch_ms'],5), r['same_box_torch_copy_ms'] and round(r['same_box_torch_copy_ms'],5))"; return 0; }
B="python3 bench.py --steps 40 --warmup 5 --cpu-seconds 0 --staged 0 --configs 0 --choco 0 --allreduce 0 --er 0"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_head.so step old$i 300 $B
  step new$i 300 $B
done
