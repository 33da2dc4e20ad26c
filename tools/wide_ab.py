"""Wide mixing kernel (65-156 slots: ER(n, 0.1) topologies with every worker on one GPU), full
rounds: per-round time from one event pair around 20 rounds, for the library in MX_GOSSIP_LIB (or the
tree's); a bit checksum of the rows after 3 rounds.  One JSON line per n.

    MX_GOSSIP_LIB=abship/lib_x.so python tools/wide_ab.py
"""
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

P = int(float(os.environ.get("WIDE_P", 2_000_000)))
for n in (72, 96, 128):
    random.seed(0)
    gp = pkg.GraphProcessor(pkg.erdos_renyi(n, 0.1, 1234), 1.0, 0, n, 4, False)
    M = len(gp.neighbors_info)
    topo = Topo(gp.neighbors_info, 0.05, np.ones((40, M), np.uint8))
    g = pkg.VirtualWorkerGroup(topo, numel=P)
    for r in range(n):
        pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[r].data_ptr(), P, 1234 + r, None))
    for j in range(3):
        g.engine.mix(j, g.layout)
    torch.cuda.synchronize()
    chk = int(g.rows[:, :P].contiguous().view(torch.int32).to(torch.int64).sum())
    for j in range(3, 8):
        g.engine.mix(j, g.layout)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(8, 28):
        g.engine.mix(j, g.layout)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 20
    print(json.dumps({"lib": os.environ.get("MX_GOSSIP_LIB") or "tree", "n": n, "M": M, "slots": g.engine.n_slots,
                      "kernel": pkg.engine.mix_kernel_name(g.engine.n_slots), "ms": round(ms, 4),
                      "TBps": round(2 * n * P * 4 / (ms * 1e-3) / 1e12, 3), "checksum": chk}), flush=True)
    g.close()
    del g
    torch.cuda.empty_cache()
