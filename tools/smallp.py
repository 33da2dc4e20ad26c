"""Small-row gossip rounds (BASELINE config 2: the repo's CIFAR ResNet, P = 181,668, 8 workers on
one GPU): mixing-kernel time per split (HIP events, median of 200) and the back-to-back round rate
through VirtualWorkerGroup.step (host launch path included)."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from conftest import Topo  # noqa: E402

n = 8
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((64, 5), np.uint8))


def events(fn, reps=200, warm=20):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


def back_to_back(fn, reps=4000):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def host_only(fn, reps=4000):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    el = time.perf_counter() - t
    torch.cuda.synchronize()
    return el / reps * 1e6


sizes = [int(x) for x in sys.argv[1:]] or [181_668, 666_547, 2_000_000, 8_000_000]
for P in sizes:
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    for i in range(n):
        pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
    B = 2 * n * P * 4
    for sp in (1, 2, 4, 0):
        pkg.engine.set_mix_tuning(split=sp)
        k_us = events(lambda: grp.engine.mix(0, grp.layout))
        r_us = back_to_back(lambda: grp.step(0))
        h_us = host_only(lambda: grp.step(0))
        # HIP graph of R device_round()s (no host work per round): GPU-side round time
        R = 50
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        grp.iter_dev.fill_(0)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g):
                for _ in range(R):
                    grp.device_round()

        def replay():
            grp.iter_dev.fill_(0)
            g.replay()
        g_us = events(replay, reps=20, warm=3) / R
        del g
        g = torch.cuda.CUDAGraph()                 # device_rounds(R): one counter launch per R rounds
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            with torch.cuda.graph(g):
                grp.device_rounds(R)
        u_us = events(replay, reps=20, warm=3) / R
        print(json.dumps({"P": P, "split": sp, "kernel_us": round(k_us, 2), "TBps": round(B / k_us / 1e6, 3),
                          "round_us_back_to_back": round(r_us, 2), "host_us_per_step": round(h_us, 2),
                          "round_us_graph": round(g_us, 2), "TBps_graph": round(B / g_us / 1e6, 3),
                          "round_us_graph_unrolled": round(u_us, 2)}), flush=True)
        del g
    pkg.engine.set_mix_tuning(split=0)
    del grp
    torch.cuda.empty_cache()
