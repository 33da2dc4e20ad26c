"""Why the launch-bound ResNet config (P = 181,668, MATCHA 0.5, graph 0) measured 8.14 us / round on
the driver's box and 5.9-6.0 us on the builder's: the same rounds host-clocked
(synchronize + wall clock around K back-to-back rounds, as bench.py's timed_loop at N = 1) for
K = 20 (the driver's --steps) / 50 (the builder's) / 400, each from an idle GPU (a 3 s host sleep,
like the CPU-baseline legs before the figure) and after a warm burst of 4000 rounds, plus per-round
HIP events (kernel time).  One JSON line.

    python tools/latency_bound.py [--params 181668]
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=181_668)
    ap.add_argument("--idle-s", type=float, default=3.0)
    args = ap.parse_args()
    pkg = importlib.import_module(PKG)
    np.random.seed(1234)
    T = 60_000
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, 8, T, True)
    g = pkg.VirtualWorkerGroup(GP, numel=args.params)
    for r in range(8):
        pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[r].data_ptr(), args.params, 1234 + r, None))
    torch.cuda.synchronize()
    it = [0]

    def rounds(K):
        for _ in range(K):
            g.step(it[0] % T)
            it[0] += 1

    def host_clocked(K):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rounds(K)
        torch.cuda.synchronize()
        return 1e6 * (time.perf_counter() - t) / K

    def events(K):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for a, b in ev:
            a.record()
            rounds(1)
            b.record()
        torch.cuda.synchronize()
        us = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
        return {"median": float(np.median(us)), "min": float(us.min()), "mean": float(us.mean())}

    out = {"params": args.params, "idle_s": args.idle_s, "cold": {}, "warm": {}}
    for K in (20, 50, 400):
        time.sleep(args.idle_s)                 # the GPU idles, as behind the bench's CPU legs
        rounds(3)                               # bench's W = 3 warmup rounds
        out["cold"][K] = {"host_us_per_round": host_clocked(K)}
        time.sleep(args.idle_s)
        rounds(4000)                            # warm burst
        out["warm"][K] = {"host_us_per_round": host_clocked(K)}
    time.sleep(args.idle_s)
    rounds(3)
    out["cold_events_400"] = events(400)
    rounds(4000)
    out["warm_events_400"] = events(400)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
