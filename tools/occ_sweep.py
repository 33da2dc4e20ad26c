"""Row kernel, 8 slots, graph 0: the plain launch (mx_mix_set spec = 0) against the SPEC form (the
round's active local rows -- the engine's host mask, mx_mix_call.need_host -- loaded before the plan
record arrives) at spec_wgpc workgroups per CU, for several row sizes, on full rounds and on a MATCHA
C_b = 0.5 schedule (BUDGET).  Per variant, interleaved REPS times: 40 back-to-back rounds between one
event pair.  Bits: 3 rounds from the same rows under every variant.  Then the centralized mean
(mx_mean_rows_to, 8 rows in place) at mean_wgpc workgroups per CU (MEANW).  One JSON line each.

    SIZES=25600000,36546980 WGPC=0,4,5,6 GLDS=0,1 BUDGET=1.0 MEANW=0,3 REPS=3 python tools/occ_sweep.py
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from conftest import Topo  # noqa: E402

L = pkg.lib
n = 8
reps = int(os.environ.get("REPS", "3"))
sizes = [int(float(x)) for x in os.environ.get("SIZES", "25600000").split(",")]
glds = [int(x) for x in os.environ.get("GLDS", "1").split(",")]   # 1: the product default
variants = [("default", None)] + [(f"spec_wgpc{w}" + ("" if gl else "_regs"), (w, gl)) for w in
                                  (int(x) for x in os.environ.get("WGPC", "0,4,5,6").split(",")) for gl in glds]
E = pkg.engine
saved = E.mix_tuning()


def setv(w):
    if w is None:
        E.set_mix_tuning(spec=0)
    else:
        E.set_mix_tuning(spec=1, spec_wgpc=w[0], spec_glds=w[1])


budget = float(os.environ.get("BUDGET", "1.0"))
if budget >= 1.0:
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    topo = Topo(gp.neighbors_info, 2 / 7, np.ones((200, len(gp.neighbors_info)), np.uint8))
else:
    np.random.seed(1234)
    topo = pkg.MatchaProcessor(pkg.select_graph(0), budget, 0, n, 200, True)
for P in sizes:
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    sums = {}
    for name, w in variants:
        setv(w)
        for r in range(n):
            pkg._lib.check(L.mx_synth_fill(grp.rows[r].data_ptr(), P, 1234 + r, None))
        for j in range(3):
            grp.engine.mix(j, grp.layout)
        torch.cuda.synchronize()
        sums[name] = int(grp.rows[:, :P].contiguous().view(torch.int32).to(torch.int64).sum())
    res = {name: [] for name, _ in variants}
    for rep in range(reps):
        for name, w in (variants if rep % 2 == 0 else variants[::-1]):
            setv(w)
            for _ in range(10):
                grp.engine.mix(0, grp.layout)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for j in range(40):
                grp.engine.mix(1 + j, grp.layout)
            b.record()
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(b) / 40)
    setv(None)
    out = {"P": P, "budget": budget, "bytes_per_full_round": 2 * n * P * 4}
    for name, _ in variants:
        ms = min(res[name])
        out[name] = {"ms_min": round(ms, 4), "ms_all": [round(x, 4) for x in res[name]],
                     "same_bits": sums[name] == sums["default"]}
    print(json.dumps(out), flush=True)
    grp.close()
    del grp
    torch.cuda.empty_cache()

meanw = [int(x) for x in os.environ.get("MEANW", "").split(",") if x]
if meanw:
    P = sizes[0]
    ld = (P + 63) // 64 * 64
    rows = torch.empty((n, ld), dtype=torch.float32, device="cuda")
    one = lambda: pkg._lib.check(L.mx_mean_rows_to(rows.data_ptr(), n, ld, P, 0, rows.data_ptr(), n, ld, None))
    res, sums = {w: [] for w in meanw}, {}
    for w in meanw:
        E.set_mix_tuning(mean_wgpc=w)
        for r in range(n):
            pkg._lib.check(L.mx_synth_fill(rows[r].data_ptr(), P, 1234 + r, None))
        one()
        torch.cuda.synchronize()
        sums[w] = int(rows[:, :P].contiguous().view(torch.int32).to(torch.int64).sum())
    for rep in range(reps):
        for w in (meanw if rep % 2 == 0 else meanw[::-1]):
            E.set_mix_tuning(mean_wgpc=w)
            for _ in range(10):
                one()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(40):
                one()
            b.record()
            torch.cuda.synchronize()
            res[w].append(a.elapsed_time(b) / 40)
    print(json.dumps({"mean_P": P, **{f"mean_wgpc{w}": {"ms_min": round(min(res[w]), 4),
                                                        "ms_all": [round(x, 4) for x in res[w]],
                                                        "frac_8TBps": round(2 * n * P * 4 / (min(res[w]) * 1e-3) / 8e12, 4),
                                                        "same_bits": sums[w] == sums[meanw[0]]} for w in meanw}}),
          flush=True)
E.set_mix_tuning(**saved)
