"""mx_mean_rows_to (the centralized all-reduce over 8 arena rows x 25.6M fp32, in place) per-launch
time over REPS repeats, next to the headline mixing kernel on the same rows in the same process;
prints the HBM fraction (2 x 8 x P x 4 bytes per launch), the kernel names and a bit checksum of the
mean.  (Round 5 used it, with knobs since removed, to A/B a persistent grid, an exact power-of-two
scale, two tiles per workgroup and compile-time row counts: profiles/r05c-f_*.log.)"""
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
L = pkg.lib
n, P = 8, int(os.environ.get("MEAN_P", 25_600_000))
ld = (P + 63) // 64 * 64
variants = ["default"]


def knobs(v):
    pass

reps = int(os.environ.get("REPS", "1"))
rows = torch.empty((n, ld), dtype=torch.float32, device="cuda")
one = lambda: pkg._lib.check(L.mx_mean_rows_to(rows.data_ptr(), n, ld, P, 0, rows.data_ptr(), n, ld, None))
res = {v: [] for v in variants}
sums = {}
for rep in range(reps):
    for v in variants:
        knobs(v)
        for r in range(n):
            pkg._lib.check(L.mx_synth_fill(rows[r].data_ptr(), P, 1234 + r, None))
        one()
        torch.cuda.synchronize()
        sums[v] = int(rows[:, :P].contiguous().view(torch.int32).to(torch.int64).sum())
        for _ in range(20):
            one()
        K = 40
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(K):
            one()
        b.record()
        torch.cuda.synchronize()
        res[v].append(a.elapsed_time(b) / K)
# the headline mixing kernel on the same rows (graph 0, every matching active), interleaved the same
# way: the same-box reference for the mean kernels' HBM rate
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import Topo  # noqa: E402
import numpy as np  # noqa: E402
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((200, len(gp.neighbors_info)), np.uint8))
grp = pkg.VirtualWorkerGroup(topo, numel=P)
mix_ms = []
for rep in range(reps):
    for _ in range(20):
        grp.engine.mix(0, grp.layout)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(40):
        grp.engine.mix(1 + j, grp.layout)
    b.record()
    torch.cuda.synchronize()
    mix_ms.append(a.elapsed_time(b) / 40)
print(json.dumps({"kernel": pkg.engine.mix_kernel_name(n), "ms_min": round(min(mix_ms), 4),
                  "ms_all": [round(x, 4) for x in mix_ms],
                  "frac_8TBps": round(2 * n * P * 4 / (min(mix_ms) * 1e-3) / 8e12, 4)}), flush=True)
for v in variants:
    ms = min(res[v])
    knobs(v)
    print(json.dumps({"variant": v, "kernel": L.mx_mean_kernel_name(rows.data_ptr(), n, ld, P, 0, rows.data_ptr(), n, ld).decode(), "ms_min": round(ms, 4),
                      "ms_all": [round(x, 4) for x in res[v]], "frac_8TBps": round(2 * n * P * 4 / (ms * 1e-3) / 8e12, 4),
                      "checksum": sums[v], "same_bits": sums[v] == sums[variants[0]]}), flush=True)
