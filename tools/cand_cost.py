"""What the Choco top-k's selection passes pay per candidate: the one-row top-k (compress only, the
VGG-16 share: P = 14,774,436, k = 147,744) on inputs whose sampled floor keeps different candidate
counts -- "uniform" (synthetic uniform[-1,1): the floor's 12-bit bin is 1/32 of the top octave wide,
~3 k candidates), "gap" (every 100th key +1000: ~1.25 k), "layers".  Median of per-call HIP events,
the candidate count from mx_topk_stats.  Env: CHOCO_P, REPS."""
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
P = int(os.environ.get("CHOCO_P", 14_774_436))
REPS = int(os.environ.get("REPS", 30))
k = max(1, int(P * 0.01))
kpad = (k + 1) // 2 * 2
x = torch.empty(P, dtype=torch.float32, device="cuda")
vals = torch.empty(kpad + 2 * k, dtype=torch.float32, device="cuda")
work = torch.zeros(int(L.mx_topk_work_bytes(P)), dtype=torch.uint8, device="cuda")


def fill(pattern):
    pkg._lib.check(L.mx_synth_fill(x.data_ptr(), P, 77, None))
    if pattern == "gap":
        x[::100] += 1000.0
    elif pattern == "gap3":                  # ~3 k candidates sitting in the floor's bin
        x[::100] += 1000.0
        x[1::100] += 1000.5
        x[2::100] += 1001.0
    elif pattern == "layers":
        e = np.linspace(0, P, 9).astype(np.int64)
        for j in range(8):
            x[e[j]:e[j + 1]] *= float(10.0 ** (j % 4 - 2))


def once():
    pkg._lib.check(L.mx_topk_abs_diff_rows(x.data_ptr(), None, P, 1, P, k, vals.data_ptr(), 0, 4 * kpad, -1,
                                           work.data_ptr(), 0, None))


out = []
for pattern in ("uniform", "gap", "gap3", "layers"):
    fill(pattern)
    for _ in range(5):
        once()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(REPS)]
    for a, b in ev:
        a.record()
        once()
        b.record()
    torch.cuda.synchronize()
    st = np.zeros(5, np.int64)
    pkg._lib.check(L.mx_topk_stats(work.data_ptr(), 0, 1, P, st.ctypes.data, None))
    us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
    r = {"pattern": pattern, "topk_us_median": round(float(np.median(us)), 2), "topk_us_min": round(float(us.min()), 2),
         "candidates": int(st[4]), "cand_per_k": round(int(st[4]) / k, 2)}
    print(json.dumps(r), flush=True)
