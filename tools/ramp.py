"""Does the headline round speed up as the GPU keeps streaming (clock / power ramp after idle)?
Back-to-back blocks of K rounds (wall clock, synchronize on both sides), consecutively, after a
1 s idle pause, three times over."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from conftest import Topo  # noqa: E402

K, BLOCKS = 20, 12
n, P = 8, 25_600_000
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((K * BLOCKS * 3 + 8, 5), np.uint8))
grp = pkg.VirtualWorkerGroup(topo, numel=P)
for i in range(n):
    pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
it = 0
for rep in range(3):
    torch.cuda.synchronize()
    time.sleep(1.0)
    for _ in range(5):
        grp.step(it)
        it += 1
    torch.cuda.synchronize()
    us = []
    for b in range(BLOCKS):
        t = time.perf_counter()
        for j in range(K):
            grp.step(it)
            it += 1
        torch.cuda.synchronize()
        us.append(round((time.perf_counter() - t) * 1e6 / K, 1))
    print(json.dumps({"after_idle": rep, "us_per_round_by_block_of_20": us}), flush=True)
