"""Choco top-k candidate floor: sampled (one sampling launch per round) vs the previous round's
exact k-th key (mx_topk_set "floor_hint" m: no sampling launch, adaptive margin starting at m bins),
under realistic drift -- x_hat catching up every round (the top-k entries of x - x_hat vanish, so
the k-th key moves down) plus an optimizer-like step between rounds (x += DRIFT * noise, the
VGG test's 0.01 x synth) -- and without drift (the bench figure).  VERDICT r03 item 3, lever 1.

One row (a rank's share at N = 8, null transport, partner messages = copies of its own) and 8 rows
(all workers on one GPU).  Per round: HIP events around the round only (the drift add is outside);
fresh groups per variant (the hint lives in the scratch); interleaved repeats; the fallback count
from mx_topk_stats.  Env: CHOCO_P, REPS, VARIANTS (s / f / h<m>, below), DRIFTS (comma list), ROUNDS,
TRACE."""
import ctypes
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
REPS = int(os.environ.get("REPS", 2))
# variants: "s" sampled digit floor (default), "f" sampled floor refined in a window (fine_floor),
# "h<m>" floor from the previous call's k-th key, margin m bins (floor_hint m)
VARIANTS = os.environ.get("VARIANTS", "s,f,h2,h4").split(",")
DRIFTS = [float(v) for v in os.environ.get("DRIFTS", "0.01,0").split(",")]
ROUNDS = int(os.environ.get("ROUNDS", 40))
TRACE = int(os.environ.get("TRACE", 0))        # 1: per round row 0's threshold key, candidates, fallbacks
WARM = 5
n = 8
GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, n, ROUNDS + WARM + 2, True)
L = pkg.lib
if os.environ.get("COMPACT_BLOCKS"):                 # compaction grid (0 = auto)
    pkg._lib.check(L.mx_topk_set(b"compact_blocks", int(os.environ["COMPACT_BLOCKS"])))


def make(kind):
    if kind == "rows8":
        c = pkg.ChocoWorkerGroup(GP, numel=P, ratio=0.99, consensus_lr=0.1)
        for i in range(n):
            pkg._lib.check(L.mx_synth_fill(c.rows[i].data_ptr(), P, 1234 + i, None))
        return c
    c = pkg.ChocoWorkerGroup(GP, numel=P, ratio=0.99, consensus_lr=0.1, rank=0, nranks=8, comm=NullComm(0, 8),
                             placement="auto")
    saved = (int(L.mx_topk_get(b"floor_hint")), int(L.mx_topk_get(b"fine_floor")))
    knobs("s")
    for s in range(c.n_local, c.engine.n_slots):      # partner stand-ins: top-k of other synthetic rows
        pkg._lib.check(L.mx_synth_fill(c.rows[0].data_ptr(), P, 7000 + s, None))
        c.compress(0)
        torch.cuda.synchronize()
        c.msgs[s * c.msg_ld:(s + 1) * c.msg_ld].copy_(c.msgs[:c.msg_ld])
    L.mx_topk_set(b"floor_hint", saved[0])
    L.mx_topk_set(b"fine_floor", saved[1])
    pkg._lib.check(L.mx_synth_fill(c.rows[0].data_ptr(), P, 1234 + c.workers[0], None))
    c.work.zero_()
    return c


def knobs(variant):
    pkg._lib.check(L.mx_topk_set(b"floor_hint", int(variant[1:]) if variant.startswith("h") else -1))
    pkg._lib.check(L.mx_topk_set(b"fine_floor", 1 if variant == "f" else 0))


def run(kind, hint, drift, noise):
    knobs(hint)
    c = make(kind)
    us, trace = [], []
    for it in range(WARM + ROUNDS):
        if drift and it:
            c.rows.add_(noise[:c.n_local], alpha=drift)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        c.step(it)
        b.record()
        torch.cuda.synchronize()
        if it >= WARM:
            us.append(a.elapsed_time(b) * 1e3)
        if TRACE:
            sr = np.zeros(5 * c.n_local, np.int64)
            pkg._lib.check(L.mx_topk_stats(c.work.data_ptr(), c.work_ld, c.n_local, c.numel, sr.ctypes.data, None))
            trace.append((float(np.uint32(sr[3]).view(np.float32)), int(sr[4]), int(sr[1])))
    if TRACE:
        print(json.dumps({"trace": kind, "drift": drift, "floor_hint": hint, "k": c.k,
                          "T_cand_fb": [(round(t, 6), cn, fb) for t, cn, fb in trace]}), flush=True)
    st = np.zeros(5 * c.n_local, np.int64)
    pkg._lib.check(L.mx_topk_stats(c.work.data_ptr(), c.work_ld, c.n_local, c.numel, st.ctypes.data, None))
    c.check_topk()
    c_k = c.k
    del c
    torch.cuda.empty_cache()
    st = st.reshape(-1, 5)
    return {"round_us_median": float(np.median(us)), "round_us_mean": float(np.mean(us)),
            "calls": int(st[:, 0].max()), "fallbacks": int(st[:, 1].sum()), "margins": st[:, 2].tolist(),
            "last_candidates_per_k": [round(int(x) / c_k, 2) for x in st[:, 4]]}


noise = torch.empty((n, P), dtype=torch.float32, device="cuda")
for i in range(n):
    pkg._lib.check(L.mx_synth_fill(noise[i].data_ptr(), P, 9000 + i, None))
res = {}
for rep in range(REPS):
    for kind in ("row1", "rows8"):
        for drift in DRIFTS:
            for hint in VARIANTS:
                r = run(kind, hint, drift, noise)
                res.setdefault((kind, drift, hint), []).append(r)
                print(json.dumps({"rep": rep, "group": kind, "drift": drift, "floor_hint": hint, **r}), flush=True)
knobs("s")
for (kind, drift, hint), rs in res.items():
    print(json.dumps({"summary": True, "group": kind, "drift": drift, "floor_hint": hint,
                      "round_us_median": round(float(np.median([r["round_us_median"] for r in rs])), 2),
                      "fallbacks_per_round": sum(r["fallbacks"] for r in rs) / max(1, sum(r["calls"] for r in rs))}))
