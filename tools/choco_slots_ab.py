"""A/B of the Choco apply pass: mx_choco_apply (messages at a fixed stride in one buffer) vs
mx_choco_apply_slots (message addresses from a device slot table, the pull transport's form; here
the table points at the same local buffer, the plan records carry the peer-reads bit so every
workgroup's system-scope acquire runs).  VGG-16 size (P = 14,774,436, top-1 %), 8 rows on one GPU
and rank 0's 4 / 2 / 1 rows of the 2 / 4 / 8-GPU layouts (received slots = top-k messages of other
synthetic rows).
Variants: strided / slot table, each without and with the peer-reads bit (the table's cost vs the
per-workgroup acquire's), the slot-table form per tile (apply_persist 0) and persistent (the
default for it: acquire and addresses once per workgroup), and the strided form persistent.  Apply launches alone, per-launch HIP events, median
of K, the variants interleaved 4 times.  One JSON line."""
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
out = {"P": P, "K": K}
for rows in (8, 4, 2, 1):
    kw = dict(numel=P, ratio=0.99, consensus_lr=0.1)
    if rows < 8:                                  # rank 0's block of the 8 // rows - GPU layout
        kw.update(rank=0, nranks=8 // rows, comm=NullComm(0, 8 // rows))
    g = pkg.ChocoWorkerGroup(topo, **kw)
    eng = g.engine
    for s in range(g.n_local, eng.n_slots):
        pkg._lib.check(L.mx_synth_fill(g.rows[0].data_ptr(), P, 7000 + s, None))
        g.compress(0)
        torch.cuda.synchronize()
        g.msgs[s * g.msg_ld:(s + 1) * g.msg_ld].copy_(g.msgs[:g.msg_ld])
    for r in range(g.n_local):
        pkg._lib.check(L.mx_synth_fill(g.rows[r].data_ptr(), P, 1234 + r, None))
    g.compress(0)
    plan_pr = eng.plan.clone()
    pkg._lib.check(L.mx_plan_set_peer_reads(plan_pr.data_ptr(), eng.T + 1, g.n_local, eng.M, 1, None))
    table = torch.tensor([g.msgs.data_ptr() + s * g.msg_ld for s in range(eng.n_slots)], dtype=torch.int64,
                         device="cuda")

    def strided(plan):
        def f(it):
            pkg._lib.check(L.mx_choco_apply(g.x.data_ptr(), g.x_hat.data_ptr(), g.s.data_ptr(), g.ld, P, g.k,
                                            g.msgs.data_ptr(), g.msg_ld, eng.n_slots, plan.data_ptr(), it,
                                            g.n_local, eng.M, eng.alpha32, g.gamma32, None, None))
        return f

    def slots(plan):
        def f(it):
            pkg._lib.check(L.mx_choco_apply_slots(g.x.data_ptr(), g.x_hat.data_ptr(), g.s.data_ptr(), g.ld, P,
                                                  g.k, table.data_ptr(), eng.n_slots, plan.data_ptr(), it,
                                                  g.n_local, eng.M, eng.alpha32, g.gamma32, None))
        return f

    def knob(fn, persist):
        def f(it):
            pkg._lib.check(L.mx_topk_set(b"apply_persist", persist))
            fn(it)
            pkg._lib.check(L.mx_topk_set(b"apply_persist", -1))
        return f

    variants = {"strided": strided(eng.plan), "strided_peer_bit": strided(plan_pr),
                "strided_persist": knob(strided(eng.plan), 1),
                "slots_peer_bit_nonpersist": knob(slots(plan_pr), 0),
                "slots": slots(eng.plan), "slots_peer_bit": slots(plan_pr)}
    res = {k: [] for k in variants}
    for rep in range(4):
        for name, fn in variants.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            for j, (a, b) in enumerate(ev):
                a.record()
                fn(j)
                b.record()
            torch.cuda.synchronize()
            res[name].append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
    out[f"rows{rows}"] = {"slots_total": int(eng.n_slots), "apply_us_median_per_rep": res,
                          **{k + "_us": float(np.median(v)) for k, v in res.items()}}
    if eng.n_slots > g.n_local:
        # mx_pull_fetch of the round's remote messages (here from this GPU's own slots: the
        # kernel's launch + acquire + copy cost without xGMI), per-launch events
        dst = torch.empty_like(g.msgs)
        rec = eng.plan.data_ptr() + 4 * 0 * eng.plan_words
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for a, b in ev:
            a.record()
            pkg._lib.check(L.mx_pull_fetch(table.data_ptr(), g.n_local, eng.n_slots - g.n_local, rec, dst.data_ptr(),
                                           g.msg_ld, g.msg_bytes, None))
            b.record()
        torch.cuda.synchronize()
        out[f"rows{rows}"]["fetch_us"] = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
        out[f"rows{rows}"]["fetch_bytes"] = int((eng.n_slots - g.n_local) * g.msg_bytes)
    del g
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
