"""Summarise FETCH_SIZE / WRITE_SIZE rocprofv3 passes of tools/choco_rounds.py into HBM bytes per
launch per kernel and per round (gfx950 corrections of MI355X_MICROARCH.md: KiB units, FETCH_SIZE
x2 for wide coalesced reads -- an upper bound for the passes' narrow candidate / message reads).

    CHOCO_GROUP=rows8 K=10 rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR/fetch -o f -- python3 tools/choco_rounds.py
    CHOCO_GROUP=rows8 K=10 rocprofv3 --pmc WRITE_SIZE --output-format csv -d DIR/write -o w -- python3 tools/choco_rounds.py
    python tools/choco_pmc.py DIR [algorithmic_bytes_per_round]"""
import collections
import csv
import glob
import json
import sys


def load(pat, cname):
    acc = collections.defaultdict(list)
    for f in glob.glob(pat, recursive=True):
        for r in csv.DictReader(open(f)):
            if (r.get("Counter_Name") or r.get("Counter-Name")) != cname:
                continue
            acc[r.get("Kernel_Name") or r.get("Kernel-Name")].append(float(r.get("Counter_Value") or r.get("Counter-Value")))
    return acc


d = sys.argv[1]
alg = float(sys.argv[2]) if len(sys.argv) > 2 else 24 * 14_774_436 * 8
F = load(d + "/fetch/**/*counter_collection.csv", "FETCH_SIZE")
W = load(d + "/write/**/*counter_collection.csv", "WRITE_SIZE")
calls = max(len(v) for v in F.values())
out, tot = {}, 0.0
for k, v in F.items():
    if len(v) < calls:                       # one-off setup kernels
        continue
    rb = 2 * 1024 * sum(v) / len(v)
    w = W.get(k, [0.0])
    wb = 1024 * sum(w) / max(1, len(w))
    out[k[:80]] = {"launches": len(v), "read_MB": rb / 1e6, "write_MB": wb / 1e6}
    tot += rb + wb
print(json.dumps({"kernels": out, "round_MB": tot / 1e6, "algorithmic_MB": alg / 1e6, "ratio": tot / alg}, indent=1))
