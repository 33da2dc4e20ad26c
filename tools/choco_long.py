"""ChocoSGD round time over many rounds without parameter drift (x_hat catches up with x, so the
magnitude distribution of x - x_hat changes round by round): 8 rows, VGG-16 size; median of each
block of 20 rounds; also with a small drift (an optimizer-like update) between rounds."""
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

P, n, B, NB = 14_774_436, 8, 20, int(os.environ.get("BLOCKS", 10))
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
for drift in (0.0, 1e-3):
    topo = Topo(gp.neighbors_info, 2 / 7, np.ones((B * NB + 2, 5), np.uint8))
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=0.99, consensus_lr=0.1)
    for i in range(n):
        pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
    noise = torch.empty((n, P), device="cuda")
    for i in range(n):
        pkg.lib.mx_synth_fill(noise[i].data_ptr(), P, 99 + i, None)
    noise.mul_(drift)
    out = []
    it = 0
    for b in range(NB):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(B)]
        for a, e in ev:
            if drift:
                grp.rows.add_(noise)
            a.record()
            grp.step(it)
            e.record()
            it += 1
        torch.cuda.synchronize()
        out.append(round(float(np.median([a.elapsed_time(e) for a, e in ev])) * 1e3, 1))
    print(json.dumps({"drift": drift, "us_per_round_by_block_of_20": out}), flush=True)
    del grp, noise
    torch.cuda.empty_cache()
