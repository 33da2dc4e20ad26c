"""Time one ChocoSGD round (top-k + scatters + dense update) for 8 workers on one GPU,
VGG-16 size (14,774,436 params, ratio 0.99 -> k = 147,744) unless overridden."""
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

P = int(os.environ.get("CHOCO_P", 14_774_436))
ratio = float(os.environ.get("CHOCO_RATIO", 0.99))
n = 8
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
K = 20
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((K + 5, 5), np.uint8))
grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1)
if os.environ.get("CHOCO_COMPACT_BLOCKS"):
    pkg._lib.check(pkg.lib.mx_topk_set(b"compact_blocks", int(os.environ["CHOCO_COMPACT_BLOCKS"])))
for i in range(n):
    pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
for it in range(5):
    grp.step(it)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
for j in range(K):
    ev[j][0].record()
    grp.step(5 + j)
    ev[j][1].record()
torch.cuda.synchronize()
ms = np.array([a.elapsed_time(b) for a, b in ev])
k = grp.k
# algorithmic bytes: top-k reads x, x_hat once (8P) per worker at minimum; scatters 12 B per
# selected element per (partner + self) read of the message + 8 B RMW of s (and x_hat for self);
# dense update reads x, s, x_hat and writes x (16P)
deg = np.zeros(n, int)
for g in range(5):
    deg += np.asarray(gp.neighbors_info[g]) >= 0
alg = int(n * (8 * P + 16 * P) + sum(int(d + 1) * k * (12 + 8) + k * 8 for d in deg))
print(json.dumps({"compact_blocks": int(pkg.lib.mx_topk_get(b"compact_blocks")), "P": P, "ratio": ratio, "k": k, "round_ms_median": float(np.median(ms)),
                  "round_ms_min": float(ms.min()), "rounds_per_s": 1e3 / float(np.median(ms)),
                  "alg_bytes_min": alg, "eff_TBps": alg / (np.median(ms) * 1e-3) / 1e12}))
