#!/bin/bash
# row kernel: 512-column sub-tiles on flat grids (8-16 slots) + flat cap 256 x 512 items: the whole
# GPU suite, then bench A/B (config figures included) against _ab/lib_s1.so, 3 interleaved repeats.
set -u
OUT=gpurun_out/r2s71; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-2} $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
B="python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --staged 0 --choco 0 --allreduce 0"
for i in 1 2 3; do
  MX_GOSSIP_LIB=_ab/lib_s1.so TAILN=0 step s1_$i 300 $B
  TAILN=0 step s2_$i 300 $B
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r2s71/s*_*.log")):
    d = json.loads([l for l in open(f) if l.startswith('{"metric"')][-1])
    c = d["configs"]
    print(f.split("/")[-1], round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["avg_launch_ms"] * 1e3, 1),
          round(d["matcha_schedule"]["rounds_per_s"]), d["parity_ok"],
          {k: round(v["ms_per_round"] * 1e3, 1) for k, v in c.items()})
PY
