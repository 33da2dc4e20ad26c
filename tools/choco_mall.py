"""Choco round A/B over mx_topk_set knob settings (VARIANTS="apply_nt=-1,apply_nt=0,compact_occ=5:
compact_blocks=1280", ":" joins knobs of one variant; "none" leaves the knobs alone, for another build
via MX_GOSSIP_LIB).  r02 builds also tried compact_nt / apply_rev (tiles last-first) and a
96-VGPR compaction (5 waves per SIMD): none helped.  8 rows on one GPU (the bench figure) and one
row (a rank's share at N = 8, null transport, received messages = valid stand-ins).  Interleaved repeats, median of per-round HIP
events.  Question asked: does the apply pass find x / x_hat in the Infinity Cache right after the
top-k pass read them (one row: 118 MB fits; 8 rows: the tails do)?"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from nullcomm import NullComm  # noqa: E402

P = int(os.environ.get("CHOCO_P", 14_774_436))
REPS = int(os.environ.get("REPS", 3))
_V = os.environ.get("VARIANTS", "apply_nt=-1,apply_nt=0,apply_nt=1")
VARIANTS = [None] if _V == "none" else _V.split(",")
n = 8
GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, n, 200, True)


DEFAULTS = {}


def setk(v):
    if v is None:
        return
    for kv in v.split(":"):
        k, x = kv.split("=")
        if k not in DEFAULTS:
            DEFAULTS[k] = int(pkg.lib.mx_topk_get(k.encode()))
        pkg._lib.check(pkg.lib.mx_topk_set(k.encode(), int(x)))


def reset():
    for k, x in DEFAULTS.items():
        pkg._lib.check(pkg.lib.mx_topk_set(k.encode(), x))


def time_rounds(c, it0, K=30):
    for j in range(5):
        c.step(it0 + j)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for j, (a, b) in enumerate(ev):
        a.record()
        c.step(it0 + 5 + j)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


groups = {}
c8 = pkg.ChocoWorkerGroup(GP, numel=P, ratio=0.99, consensus_lr=0.1)
for i in range(n):
    pkg._lib.check(pkg.lib.mx_synth_fill(c8.rows[i].data_ptr(), P, 1234 + i, None))
groups["rows8"] = c8
c1 = pkg.ChocoWorkerGroup(GP, numel=P, ratio=0.99, consensus_lr=0.1, rank=0, nranks=8, comm=NullComm(0, 8),
                          placement="auto")
for s in range(c1.n_local, c1.engine.n_slots):      # partner stand-ins: top-k of other synthetic rows
    pkg._lib.check(pkg.lib.mx_synth_fill(c1.rows[0].data_ptr(), P, 7000 + s, None))
    c1.compress(0)
    torch.cuda.synchronize()
    c1.msgs[s * c1.msg_ld:(s + 1) * c1.msg_ld].copy_(c1.msgs[:c1.msg_ld])
pkg._lib.check(pkg.lib.mx_synth_fill(c1.rows[0].data_ptr(), P, 1234 + c1.workers[0], None))
c1.work.zero_()
groups["row1"] = c1

res = {(g, v): [] for g in groups for v in VARIANTS}
it = 0
for rep in range(REPS):
    for g, c in groups.items():
        for v in VARIANTS:
            reset()
            setk(v)
            res[(g, v)].append(time_rounds(c, it % 150))
            it += 40
            print(json.dumps({"rep": rep, "group": g, "variant": v,
                              "round_us": round(res[(g, v)][-1], 2)}), flush=True)
reset()
for (g, v), xs in res.items():
    print(json.dumps({"group": g, "variant": v,
                      "round_us_min": round(min(xs), 2), "round_us_median": round(float(np.median(xs)), 2)}))
