"""Config 5's per-GPU mixing work measured on ONE GPU: the ER(64, 0.1, 1234)
topology's worker shares at N = 8 / 4 / 2 (placement "auto", as bench.py) with a null transport
(the exchange is skipped; slab rows hold stand-in data) and the whole 64-row round at N = 1,
every matching active.  The mixing kernel alone is timed per share (HIP events, median) for each
knob variant; HBM rate on the algorithmic bytes (2 x active local rows + received slab rows) x P x 4,
beside the 8-slot headline kernel on the same box.

    ER_P=250000000 VARIANTS="base;ns48=1;ns48=1,blocks_per_cu=3" python tools/er_share.py
"""
import importlib
import json
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
E = pkg.engine


class NullComm:
    def __init__(self, rank, nranks):
        self.rank, self.nranks, self.handle = rank, nranks, None

    def exchange_round(self, engine, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes):
        return 0


def ev_ms(fn, reps=10, warm=3):
    for j in range(warm):
        fn(j)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for j, (a, b) in enumerate(ev):
        a.record()
        fn(warm + j)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def variants():
    out = []
    for v in os.environ.get("VARIANTS", "base").split(";"):
        kn = {}
        if v and v != "base":
            for kv in v.split(","):
                k, x = kv.split("=")
                kn[k] = int(x)
        out.append((v or "base", kn))
    return out


def main():
    P = int(float(os.environ.get("ER_P", 2.5e8)))
    Ns = [int(x) for x in os.environ.get("ER_NS", "8,4,2,1").split(",")]
    n, T = 64, 40
    random.seed(0)
    base = pkg.erdos_renyi(n, 0.1, 1234)
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(base, 1.0, 0, n, T, False)
    default = E.mix_tuning()
    # reference on the same box: the headline's 8-slot kernel, 8 x 25.6M
    np.random.seed(1234)
    GH = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, 8, T, True)
    gh = pkg.VirtualWorkerGroup(GH, numel=25_600_000)
    for r in range(8):
        pkg._lib.check(pkg.lib.mx_synth_fill(gh.rows[r].data_ptr(), gh.numel, 1234 + r, None))
    hms = ev_ms(lambda it: gh.engine.mix(it, gh.layout), 20)
    print(json.dumps({"headline_8slot_us": 1e3 * hms, "headline_TBps": 1.6384e9 / hms / 1e9}), flush=True)
    del gh
    torch.cuda.empty_cache()
    for N in Ns:
        blocks = E.partition(n, N)
        # the busiest share: the rank with the most slots
        best = None
        for r in range(N):
            topo, perm = pkg.placement.place(GP, N, "auto" if N > 1 else None)
            part = np.asarray(topo.neighbors_info, np.int32).reshape(-1, n)
            rb, nl = blocks[r]
            slots = nl + E.max_incoming_remote(part, rb, nl)
            if best is None or slots > best[1]:
                best = (r, slots)
        r = best[0]
        comm = NullComm(r, N) if N > 1 else None
        g = pkg.VirtualWorkerGroup(GP, numel=P, rank=r, nranks=N, comm=comm, placement="auto" if N > 1 else None)
        for i in range(g.n_local):
            pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[i].data_ptr(), P, 1234 + g.workers[i], None))
        if g.slab is not None:
            g.slab.fill_(0.5)
        eng = g.engine
        flags = np.ones((1, eng.M), np.uint8)
        hbm = float(_bytes(eng, flags, r, g, P)[0][0])
        for name, kn in variants():
            E.set_mix_tuning(**default)
            E.set_mix_tuning(**kn)
            lay = E.Layout([g.numel], [[p] for p in g._row_ptrs] +
                           ([[g.slab[k].data_ptr()] for k in range(eng.max_remote)] if g.slab is not None else []),
                           eng.n_slots)
            ms = ev_ms(lambda it: eng.mix(it, lay))
            print(json.dumps({"N": N, "rank": r, "slots": int(eng.n_slots), "local_rows": g.n_local,
                              "remote": int(eng.max_remote), "P": P, "variant": name,
                              "kernel": E.mix_kernel_name(eng.n_slots), "us": 1e3 * ms,
                              "TBps": hbm / (ms * 1e-3) / 1e12, "frac": hbm / (ms * 1e-3) / 8e12,
                              "vs_headline": (hbm / ms) / (1.6384e9 / hms)}), flush=True)
        E.set_mix_tuning(**default)
        g.close()
        del g
        torch.cuda.empty_cache()


def _bytes(eng, flags, rank, g, P):
    sys.path.insert(0, ROOT)
    import bench
    return bench.round_bytes(eng.partner, eng.owner, flags, rank, g.row_base, g.n_local, P)


if __name__ == "__main__":
    main()
