"""Row kernel sub-tiles (split 1 / 2) x grid (GRAPH = topology id: 0 = 8 workers, 2 = 16) (persistent: flat_small 0 / one workgroup per item:
flat_small 256) on 8 workers x P, graph 0, every matching active.  Mixing kernel HIP events,
median of 60, 3 interleaved repeats."""
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

GRAPH = os.environ.get("GRAPH", "0")
if GRAPH.startswith("er"):               # er<n>: ER(n, 0.1), host decomposition (widebench's graphs)
    import random
    random.seed(0)
    n = int(GRAPH[2:])
    gp = pkg.GraphProcessor(pkg.erdos_renyi(n, 0.1, 1234), 1.0, 0, n, 4, False)
else:
    n = pkg.GRAPH_SIZES[int(GRAPH)]
    gp = pkg.GraphProcessor(pkg.select_graph(int(GRAPH)), 1.0, 0, n, 4, True)
M = len(gp.neighbors_info)
topo = Topo(gp.neighbors_info, 1.0 / (M + 1), np.ones((8, M), np.uint8))
sizes = [int(x) for x in os.environ.get("SIZES", "2000000,4000000,8000000,25600000,36546980").split(",")]
variants = [tuple(int(y) for y in v.split(":")) for v in os.environ.get("VARIANTS", "1:0,1:256,2:0,2:256").split(",")]
NT = [int(x) for x in os.environ.get("NT", "1").split(",")]   # nontemporal hint settings to cross with


def kernel_us(grp, reps=60):
    for _ in range(10):
        grp.engine.mix(0, grp.layout)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        grp.engine.mix(0, grp.layout)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


saved = pkg.engine.mix_tuning()
for P in sizes:
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    for i in range(n):
        pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
    res = {(v, nt): [] for v in variants for nt in NT}
    for rep in range(3):
        for (sp, fl), nt in res:
            pkg.engine.set_mix_tuning(split=sp, flat_small=fl, nontemporal=nt)
            res[((sp, fl), nt)].append(kernel_us(grp))
    pkg.engine.set_mix_tuning(**saved)
    for ((sp, fl), nt), xs in res.items():
        us = float(np.median(xs))
        print(json.dumps({"graph": GRAPH, "P": P, "split": sp, "flat_small": fl, "nontemporal": nt, "kernel_us": round(us, 1),
                          "TBps": round(2 * n * P * 4 / us / 1e6, 3)}), flush=True)
    del grp
    torch.cuda.empty_cache()
