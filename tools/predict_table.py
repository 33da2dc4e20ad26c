"""The expected N > 1 round of every exchange form, from its measured / computed parts (DESIGN.md §6
table) -- on ONE GPU, before any multi-GPU node has run the bench.

Graph 0, 8 workers x P fp32 (default the headline's 25.6M), every matching active, placement
"auto" (bench.py's default).  For N = 2 / 4 / 8 and every rank: the rank's share of the layout is
built with a null transport (tools/nullcomm.py: no transfer; received rows hold stand-ins), and its
mixing kernel alone is timed (HIP events, median of K launches) -- the "mixing share" term.  The
busiest directed link's bytes per round come from bench.round_bytes; bench.predict_round adds the
form's fixed cost (pull measured, RCCL assumed) and, for pull, the snapshot copy.  The slowest
rank's mixing time is used (the round ends with it).  Then the same for ChocoSGD rounds (config 4:
compress + apply per rank, the busiest link's messages, bench.predict_choco).  Prints two JSON
lines."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import bench  # noqa: E402
from nullcomm import NullComm  # noqa: E402

pkg = importlib.import_module(bench.PKG_NAME)
P = int(float(os.environ.get("PRED_P", 25_600_000)))
K = int(os.environ.get("K", 20))
n = 8
np.random.seed(1234)
GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, n, K + 8, True)
out = {"graph": 0, "workers": n, "P": P, "placement": "auto", "rows": []}
for N in (2, 4, 8):
    mix, links, pubs, slots = [], [], [], []
    for r in range(N):
        g = pkg.VirtualWorkerGroup(GP, numel=P, rank=r, nranks=N, comm=NullComm(r, N), placement="auto")
        for i in range(g.n_local):
            pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[i].data_ptr(), P, 1234 + g.workers[i], None))
        for j in range(3):
            g.engine.mix(j, g.layout)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for j, (a, b) in enumerate(ev):
            a.record()
            g.engine.mix(3 + j, g.layout)
            b.record()
        torch.cuda.synchronize()
        mix.append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e-3)
        flags = np.asarray(GP.active_flags[3:3 + K], np.uint8)
        hbm, link, _, _ = bench.round_bytes(g.engine.partner, g.engine.owner, flags, r, g.row_base, g.n_local, P)
        links.append(float(np.mean(link)))
        pubs.append(2 * g.n_local * P * 4)
        slots.append(int(g.engine.n_slots))
        del g
        torch.cuda.empty_cache()
    mix_s, lb, pub = max(mix), max(links), max(pubs)
    row = {"N": N, "slots_per_rank": slots, "mix_ms_per_rank": [round(1e3 * m, 4) for m in mix],
           "busiest_link_bytes": lb}
    for form in ("rccl", "rccl_chunked", "pull"):
        row[form] = bench.predict_round(form, N, lb, mix_s, pub, 4, "one-GPU mixing share of the slowest rank")
    out["rows"].append(row)
print(json.dumps(out), flush=True)

# ChocoSGD (config 4: VGG-16 size, top-1 %): every rank's compress + apply with the null transport
# (received message slots hold stand-ins: the top-k messages of other synthetic rows, as the bench's
# one-row share), per-round HIP events, median; link bytes = the busiest link's messages
CP = int(float(os.environ.get("PRED_CHOCO_P", 14_774_436)))
cout = {"graph": 0, "workers": n, "P": CP, "ratio": 0.99, "placement": "auto", "rows": []}
for N in (2, 4, 8):
    loc, links, pubs = [], [], []
    for r in range(N):
        c = pkg.ChocoWorkerGroup(GP, numel=CP, ratio=0.99, consensus_lr=0.1, rank=r, nranks=N, comm=NullComm(r, N),
                                 placement="auto")
        for s in range(c.n_local, c.engine.n_slots):
            pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[0].data_ptr(), CP, 7000 + s, None))
            c.compress(0)
            torch.cuda.synchronize()
            c.msgs[s * c.msg_ld:(s + 1) * c.msg_ld].copy_(c.msgs[:c.msg_ld])
        for i in range(c.n_local):
            pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[i].data_ptr(), CP, 1234 + c.workers[i], None))
        c.work.zero_()
        for j in range(3):
            c.step(j)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for j, (a, b) in enumerate(ev):
            a.record()
            c.step(3 + j)
            b.record()
        torch.cuda.synchronize()
        loc.append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e-3)
        flags = np.asarray(GP.active_flags[3:3 + K], np.uint8)
        _, link, _, _ = bench.round_bytes(c.engine.partner, c.engine.owner, flags, r, c.row_base, c.n_local,
                                          c.msg_bytes / 4)
        links.append(float(np.mean(link)))
        pubs.append(c.n_local * c.msg_ld)
        del c
        torch.cuda.empty_cache()
    row = {"N": N, "local_ms_per_rank": [round(1e3 * v, 4) for v in loc], "busiest_link_bytes": max(links)}
    for form in ("rccl", "pull"):
        row[form] = bench.predict_choco(form, N, max(links), max(loc), max(pubs))
    cout["rows"].append(row)
print(json.dumps(cout), flush=True)
