"""Does a warm Infinity Cache (MALL) speed up the Choco apply of ONE row (config 4's per-GPU share
at N = 8)?  The apply pass alone (mx_choco_apply, messages already in place), per-launch HIP events,
median of K, after one of:
  cold  -- a 1 GB unrelated buffer read right before (evicts the rows from the 256 MB MALL)
  s     -- s read right before (torch sum)
  all   -- x, x_hat and s read right before
(the reads are outside the timed launch).  One JSON line."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402
from conftest import Topo  # noqa: E402
from nullcomm import NullComm  # noqa: E402

pkg = importlib.import_module(bench.PKG_NAME)
L = pkg.lib
P = int(float(os.environ.get("P", 14_774_436)))
K = int(os.environ.get("K", 20))
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
M = len(gp.neighbors_info)
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((K + 8, M), np.uint8))
g = pkg.ChocoWorkerGroup(topo, numel=P, ratio=0.99, consensus_lr=0.1, rank=0, nranks=8, comm=NullComm(0, 8),
                         placement="auto")
eng = g.engine
for s in range(g.n_local, eng.n_slots):
    pkg._lib.check(L.mx_synth_fill(g.rows[0].data_ptr(), P, 7000 + s, None))
    g.compress(0)
    torch.cuda.synchronize()
    g.msgs[s * g.msg_ld:(s + 1) * g.msg_ld].copy_(g.msgs[:g.msg_ld])
pkg._lib.check(L.mx_synth_fill(g.rows[0].data_ptr(), P, 1234, None))
g.compress(0)
flush = torch.ones(256 * 1024 * 1024, dtype=torch.float32, device="cuda")     # 1 GB
sink = torch.zeros(4, dtype=torch.float32, device="cuda")


def apply(it):
    pkg._lib.check(L.mx_choco_apply(g.x.data_ptr(), g.x_hat.data_ptr(), g.s.data_ptr(), g.ld, P, g.k,
                                    g.msgs.data_ptr(), g.msg_ld, eng.n_slots, eng.plan.data_ptr(), it,
                                    g.n_local, eng.M, eng.alpha32, g.gamma32, None, None))


prep = {"cold": lambda: sink[0].copy_(flush.sum()),
        "s": lambda: (sink[0].copy_(flush.sum()), sink[1].copy_(g.s.sum())),
        "all": lambda: (sink[0].copy_(flush.sum()), sink[1].copy_(g.s.sum()), sink[2].copy_(g.x.sum()),
                        sink[3].copy_(g.x_hat.sum()))}
res = {k: [] for k in prep}
for rep in range(3):
    for name, fn in prep.items():
        ts = []
        for j in range(K):
            fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            apply(j % 4)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[name].append(float(np.median(ts)))
print(json.dumps({"P": P, "K": K, "apply_us_per_rep": res, **{k + "_us": float(np.median(v)) for k, v in res.items()},
                  "apply_nt": int(L.mx_topk_get(b"apply_nt"))}), flush=True)
