#!/bin/bash
# row kernel: one workgroup per work item for rounds up to 128 x 512 items (headline and WRN-28-10
# included) vs up to 4 x 512 (_ab/lib_f4.so): bench A/B with the config figures, 3 interleaved repeats.
set -u
OUT=gpurun_out/r2s65; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi; return 0; }
B="python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --staged 0 --choco 0 --allreduce 0"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_f4.so step f4_$i 300 $B
  step f128_$i 300 $B
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r2s65/f*.log")):
    d = json.loads([l for l in open(f) if l.startswith('{"metric"')][-1])
    c = d["configs"]
    print(f.split("/")[-1], round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["avg_launch_ms"] * 1e3, 1),
          {k: round(v["ms_per_round"] * 1e3, 1) for k, v in c.items()})
PY
