"""mx_mean_rows_to (the centralized all-reduce over 8 arena rows x 25.6M fp32, in place) per-launch
time of the library it loads (MX_GOSSIP_LIB selects another build for an A/B; the geometry
experiments it timed are in profiles/r04b_mean_rows_geometry.log, r04w_*, r04ac_*); prints the HBM
fraction (2 x 8 x P x 4 bytes per launch) and a checksum of the result."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
L = pkg.lib
n, P = 8, int(os.environ.get("MEAN_P", 25_600_000))
ld = (P + 63) // 64 * 64
rows = torch.empty((n, ld), dtype=torch.float32, device="cuda")
for r in range(n):
    pkg._lib.check(L.mx_synth_fill(rows[r].data_ptr(), P, 1234 + r, None))
one = lambda: pkg._lib.check(L.mx_mean_rows_to(rows.data_ptr(), n, ld, P, 0, rows.data_ptr(), n, ld, None))
one()
torch.cuda.synchronize()
chk = float(rows[:, :P].double().sum())
for _ in range(20):
    one()
K = 40
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(K):
    one()
b.record()
torch.cuda.synchronize()
ms = a.elapsed_time(b) / K
print(json.dumps({"lib": os.environ.get("MX_GOSSIP_LIB") or "tree", "ms": round(ms, 4),
                  "frac_8TBps": round(2 * n * P * 4 / (ms * 1e-3) / 8e12, 4), "checksum": chk}), flush=True)
