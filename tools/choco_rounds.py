"""K Choco rounds of one group (CHOCO_GROUP = rows8: 8 rows on one GPU; row1: one row, a rank's
share at N = 8 with a null transport) -- a short fixed workload for rocprofv3 kernel traces; prints
the per-round HIP-event median / min (us) of the last K - 5 rounds as one JSON line (same-box A/B
of library builds through MX_GOSSIP_LIB)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from nullcomm import NullComm  # noqa: E402

P = int(os.environ.get("CHOCO_P", 14_774_436))
K = int(os.environ.get("K", 30))
GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, 8, K + 10, True)
if os.environ.get("CHOCO_GROUP", "row1") == "rows8":
    c = pkg.ChocoWorkerGroup(GP, numel=P, ratio=0.99, consensus_lr=0.1)
    for i in range(8):
        pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[i].data_ptr(), P, 1234 + i, None))
else:
    c = pkg.ChocoWorkerGroup(GP, numel=P, ratio=0.99, consensus_lr=0.1, rank=0, nranks=8, comm=NullComm(0, 8),
                             placement="auto")
    for s in range(c.n_local, c.engine.n_slots):      # partner stand-ins: top-k of other synthetic rows
        pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[0].data_ptr(), P, 7000 + s, None))
        c.compress(0)
        torch.cuda.synchronize()
        c.msgs[s * c.msg_ld:(s + 1) * c.msg_ld].copy_(c.msgs[:c.msg_ld])
    pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[0].data_ptr(), P, 1234 + c.workers[0], None))
    c.work.zero_()
for kv in filter(None, os.environ.get("TOPK_SET", "").split(":")):     # e.g. TOPK_SET=select=1:select_blocks=32
    k_, v_ = kv.split("=")
    pkg._lib.check(pkg.lib.mx_topk_set(k_.encode(), int(v_)))
import json  # noqa: E402
ev = []
for it in range(K):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    c.step(it)
    b.record()
    ev.append((a, b))
torch.cuda.synchronize()
us = sorted(1e3 * a.elapsed_time(b) for a, b in ev[5:])
print(json.dumps({"group": os.environ.get("CHOCO_GROUP", "row1"), "lib": os.environ.get("MX_GOSSIP_LIB") or "tree",
                  "topk_set": os.environ.get("TOPK_SET", ""),
                  "rounds": len(us), "round_us_median": round(us[len(us) // 2], 2), "round_us_min": round(us[0], 2)}),
      flush=True)
