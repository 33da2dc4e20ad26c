"""BASELINE config 5 on ONE MI355X: a 64-worker Erdos-Renyi topology, P parameters per worker
(default 1e9 -> a 256 GB worker arena in HBM), MATCHA budget sweep 0.1 .. 1.0.

Per budget: MatchaProcessor (host solver, GPU flags) on the same decomposition, K timed rounds
of the in-place mixing kernel over all 64 rows, rounds/s and HBM GB/s (algorithmic bytes
2 * active rows * P * 4 per round).  Parity at this size is checked without copying the arena
back: before one round per budget a fixed set of 64 columns of every row is snapshotted, the
oracle runs that round on the snapshot, and the GPU's columns must match bit-exactly.

    python tools/er_sweep.py [P] [K]
"""
import importlib
import json
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
import oracle as O  # noqa: E402

P = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
n, p_edge, seed = 64, 0.1, 1234
BUDGETS = [0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0]

random.seed(0)
base = pkg.erdos_renyi(n, p_edge, seed)
np.random.seed(seed)
t0 = time.time()
GP0 = pkg.MatchaProcessor(base, 1.0, 0, n, K + 2, False)
sub = GP0.subGraphs
M = len(sub)
print(json.dumps({"graph": f"ER({n}, {p_edge}, seed {seed})", "edges": sum(len(m) for m in sub), "matchings": M,
                  "P": P, "arena_GB": n * P * 4 / 1e9}), flush=True)
group = pkg.VirtualWorkerGroup(GP0, numel=P)
for r in range(n):
    pkg._lib.check(pkg.lib.mx_synth_fill(group.rows[r].data_ptr(), P, 1234 + r, None))
torch.cuda.synchronize()
cols = torch.from_numpy(np.linspace(0, P - 1, 64).astype(np.int64)).cuda()
partner = np.asarray(GP0.neighbors_info, np.int32)

for b in BUDGETS:
    np.random.seed(seed)
    GP = pkg.MatchaProcessor(sub, b, 0, n, K + 2, True)          # same matchings, budget b
    assert np.array_equal(np.asarray(GP.neighbors_info, np.int32), partner)
    group.engine = pkg.GossipEngine(GP, 0, n)
    group.topology = GP
    flags = np.asarray(GP.active_flags, np.uint8)
    # parity round (iteration 0)
    snap = group.rows.index_select(1, cols).cpu().numpy()
    group.step(0)
    got = group.rows.index_select(1, cols).cpu().numpy()
    want = O.decen_round(np.ascontiguousarray(snap), partner, flags[0], GP.neighbor_weight) \
        if flags[0].any() else snap
    exact = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    # timed rounds
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    t = time.perf_counter()
    for j in range(K):
        ev[j][0].record()
        group.step(1 + j)
        ev[j][1].record()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    ms = [a.elapsed_time(c) for a, c in ev]
    byts = []
    for f in flags[1:1 + K]:
        deg = np.zeros(n, int)
        for g in range(M):
            if f[g]:
                deg += partner[g] >= 0
        byts.append(2 * int((deg > 0).sum()) * P * 4)
    act = [a for a, m in zip(byts, ms) if a]
    print(json.dumps({"budget": b, "p": [round(float(x), 4) for x in GP.probabilities],
                      "alpha": GP.neighbor_weight, "rounds_per_s": K / el,
                      "mean_active_matchings": float(flags[1:1 + K].sum(1).mean()),
                      "hbm_TBps": (sum(act) / 1e12) / (sum(m for a, m in zip(byts, ms) if a) * 1e-3) if act else None,
                      "parity_64_columns_bit_exact": exact}), flush=True)
print(json.dumps({"total_s": time.time() - t0}))
