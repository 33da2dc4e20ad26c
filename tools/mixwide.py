"""Mixing-kernel throughput on the wide-slot layouts (16 / 32 / 64 workers on one GPU), full rounds,
same arena bytes as the headline (about 819 MB of rows), against torch copy_ of the same bytes."""
import importlib
import json
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from conftest import Topo  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


TOTAL = int(os.environ.get("MIXWIDE_TOTAL", 8 * 25_600_000))
if os.environ.get("MIXWIDE_TUNE"):
    KEYS = ("blocks_per_cu", "unroll", "nontemporal", "prefetch", "regidx", "chunked", "grid", "readlane_min", "rows")
    pkg.engine.set_mix_tuning(**dict(zip(KEYS, (int(v) for v in os.environ["MIXWIDE_TUNE"].split(",")))))
print(json.dumps({"tuning": pkg.engine.mix_tuning()}))
cases = [("graph0", 8, None), ("graph2", 16, None), ("er32", 32, 0.2), ("er64", 64, 0.1)]
for name, n, p in cases:
    random.seed(0)
    if p is None:
        gid = 0 if name == "graph0" else 2
        gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    else:
        gp = pkg.GraphProcessor(pkg.erdos_renyi(n, p, 1234), 1.0, 0, n, 4, False)
    M = len(gp.neighbors_info)
    topo = Topo(gp.neighbors_info, 0.05, np.ones((4, M), np.uint8))
    P = TOTAL // n
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    for i in range(n):
        pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
    part = np.asarray(gp.neighbors_info)
    act = int(((part >= 0).sum(0) > 0).sum())
    byts = 2 * act * P * 4
    ms = timeit(lambda: grp.engine.mix(0, grp.layout))
    print(json.dumps({"case": name, "n": n, "M": M, "P": P, "tile": grp.layout.tile, "us": ms * 1e3,
                      "TBps": byts / ms / 1e9}), flush=True)
    del grp
    torch.cuda.empty_cache()
src = torch.empty(TOTAL, device="cuda")
dst = torch.empty_like(src)
ms = timeit(lambda: dst.copy_(src))
print(json.dumps({"case": "torch copy_", "us": ms * 1e3, "TBps": 2 * TOTAL * 4 / ms / 1e9}))
