"""Row stride of the worker arena vs the headline round: 8 rows of P = 25.6M fp32 with ld = P +
pad floats (pad 0 = the engine's ld), graph 0, every matching active, same kernel and bytes through
the pointer-table layout.  Per-round HIP events, median of 60 rounds, 3 interleaved repeats."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from conftest import Topo  # noqa: E402

n, P = 8, 25_600_000
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
M = len(gp.neighbors_info)
K = 60
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((K + 10, M), np.uint8))
eng = pkg.GossipEngine(topo)
PADS = [int(x) for x in os.environ.get("PADS", "0,64,256,1024,4096,16384,65536,263168").split(",")]
arena = torch.empty(n * (P + max(PADS)), dtype=torch.float32, device="cuda")
base = arena.data_ptr()
for r in range(n):
    pkg._lib.check(pkg.lib.mx_synth_fill(base + 4 * r * P, P, 1234 + r, None))


def rounds(lay):
    for j in range(5):
        eng.mix(j, lay)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for j, (a, b) in enumerate(ev):
        a.record()
        eng.mix(5 + j, lay)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


lays = {p: pkg.Layout([P], [[base + 4 * r * (P + p)] for r in range(n)], eng.n_slots) for p in PADS}
res = {p: [] for p in PADS}
for rep in range(3):
    for p in PADS:
        res[p].append(rounds(lays[p]))
        print(json.dumps({"rep": rep, "pad_floats": p, "round_us": round(res[p][-1], 1)}), flush=True)
for p in PADS:
    print(json.dumps({"pad_floats": p, "row_stride_bytes": 4 * (P + p), "round_us_min": round(min(res[p]), 1),
                      "round_us_median": round(float(np.median(res[p])), 1)}))
