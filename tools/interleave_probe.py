"""Does the distance between the 8 rows a mixing tile reads matter?  The headline round (graph 0,
8 workers x 25.6M fp32, every matching active) timed on the standard arena (8 contiguous rows,
102 MB apart) and on arenas split into S segments [S][8][P/S] (the 8 rows of a segment P/S*4 bytes
apart, the segments one after another) through the pointer-table layout -- same kernel, same bytes,
same results (checked on sampled columns).  Per-round HIP events, median of 60 rounds, repeated."""
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
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((4 * K + 20, M), np.uint8))
eng = pkg.GossipEngine(topo)
arena = torch.empty(n * P, dtype=torch.float32, device="cuda")
for r in range(n):
    pkg._lib.check(pkg.lib.mx_synth_fill(arena.data_ptr() + 4 * r * P, P, 1234 + r, None))
base = arena.data_ptr()


def layout(S):
    """S segments; segment s holds columns [s*L, (s+1)*L) of every row, rows L*4 bytes apart"""
    if S == 0:                       # standard arena: row r contiguous at r*P
        return pkg.Layout([P], [[base + 4 * r * P] for r in range(n)], eng.n_slots)
    L = P // S
    lens = [L] * S
    ptrs = [[base + 4 * (s * n * L + r * L) for s in range(S)] for r in range(n)]
    return pkg.Layout(lens, ptrs, eng.n_slots)


def rounds(lay, it0):
    for j in range(5):
        eng.mix(it0 + j, lay)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for j, (a, b) in enumerate(ev):
        a.record()
        eng.mix(it0 + 5 + j, lay)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


variants = [0, 25, 100, 250, 1000, 5000]
lays = {S: layout(S) for S in variants}
res = {S: [] for S in variants}
for rep in range(3):
    for S in variants:
        res[S].append(rounds(lays[S], 0))      # the same K flags every time (all matchings active)
        print(json.dumps({"rep": rep, "segments": S, "round_us": round(res[S][-1], 1)}), flush=True)
for S in variants:
    print(json.dumps({"segments": S, "rows_apart_MB": (P if S == 0 else P // S) * 4 / 1e6,
                      "round_us_min": round(min(res[S]), 1), "round_us_median": round(float(np.median(res[S])), 1)}))
