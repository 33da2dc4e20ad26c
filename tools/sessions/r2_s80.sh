#!/bin/bash
# row kernel nontemporal = auto (ordinary accesses when the rows fit in the Infinity Cache):
# whole GPU suite, then tools/smallp.py and the headline bench on both builds (same box).
set -u
OUT=gpurun_out/r2s80; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc"; tail -${TAILN:-2} $OUT/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then exit $rc; fi; return 0; }
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
for i in 1 2; do
  MX_GOSSIP_LIB=_ab/lib_ntfixed.so TAILN=0 step old$i 300 python -u tools/smallp.py 181668 666547 2000000 8000000
  TAILN=0 step new$i 300 python -u tools/smallp.py 181668 666547 2000000 8000000
done
grep -h '"split": 0' $OUT/old1.log $OUT/new1.log $OUT/old2.log $OUT/new2.log | cut -c1-140
B="python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --staged 0 --choco 0 --allreduce 0"
MX_GOSSIP_LIB=_ab/lib_ntfixed.so TAILN=0 step bench_old 300 $B
TAILN=0 step bench_new 300 $B
python - <<'PY'
import json
for f in ("bench_old", "bench_new"):
    d = json.loads([l for l in open(f"gpurun_out/r2s80/{f}.log") if l.startswith('{"metric"')][-1])
    print(f, round(d["ms_per_step"] * 1e3, 1), d["parity_ok"], {k: round(v["ms_per_round"] * 1e3, 2) for k, v in d["configs"].items()})
PY
