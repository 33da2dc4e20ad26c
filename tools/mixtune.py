"""Sweep mixing-kernel tunings on the headline shape (8 workers x 25.6M, graph 0, full rounds)."""
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

n, P = 8, int(os.environ.get("MIXTUNE_P", 25_600_000))
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((4, 5), np.uint8))
grp = pkg.VirtualWorkerGroup(topo, numel=P)
for i in range(n):
    pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
BYTES = 2 * n * P * 4


def timeit(fn, reps=40, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    return float(np.median(ms)), float(ms.min())


KEYS = ("blocks_per_cu", "unroll", "nontemporal", "prefetch", "regidx", "chunked", "grid", "readlane_min", "rows", "split")
configs = []
for spec in sys.argv[1:] or ["sweep"]:
    if spec == "sweep":
        for rg, pf in ((0, 0), (0, 1), (1, 0), (1, 1)):
            for ch in (0, 1):
                for bpc in (3, 4, 5, 6, 8):
                    configs.append((bpc, 1, 1, pf, rg, ch, 0))
    else:
        cfg = tuple(int(x) for x in spec.split(","))
        configs.append(cfg)
DEFAULT_TAIL = (0, 32, 1, 0)   # grid, readlane_min, rows, split
configs = [c + DEFAULT_TAIL[len(c) - len(KEYS):] if len(c) < len(KEYS) else c for c in configs]
src = torch.empty((n, P), device="cuda")
dst = torch.empty_like(src)
refs = []
med, mn = timeit(lambda: dst.copy_(src))
refs.append(med)
res = []
for cfg in configs:
    pkg.engine.set_mix_tuning(**dict(zip(KEYS, cfg)))
    lay = pkg.Layout([P], [[grp.arena[r].data_ptr()] for r in range(n)], grp.engine.n_slots)
    med, mn = timeit(lambda: grp.engine.mix(0, lay))
    res.append({"cfg": "bpc=%d U=%d NT=%d PF=%d REG=%d CH=%d GRID=%d RL=%d ROWS=%d SPLIT=%d" % cfg, "med_us": med * 1e3, "min_us": mn * 1e3,
                "TBps": BYTES / med / 1e9, "frac": BYTES / med / 1e9 / 8.0})
    print(json.dumps(res[-1]), flush=True)
med, mn = timeit(lambda: dst.copy_(src))
refs.append(med)
print(json.dumps({"cfg": "torch copy_ (same bytes), before/after", "med_us": [r * 1e3 for r in refs],
                  "TBps": [BYTES / r / 1e9 for r in refs]}))
best = min(res, key=lambda r: r["med_us"])
print("BEST", json.dumps(best))
