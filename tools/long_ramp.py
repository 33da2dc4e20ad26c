"""Does the headline round keep getting faster past the bench's 50 ms settle?  The graph-0 headline
group (8 workers x 25.6M fp32, every matching active), rounds back to back for --seconds, one HIP
event pair per block of 100 rounds; prints per block the wall time since the start and the mean
round time.  One JSON line.  (round 6: the same box measured 0.2757 ms/step in a bench run and
0.2597 in the rocprofv3 run that followed it -- profiles/r06e_bench.json, r06_bench_under_rocprof.json.)

    python tools/long_ramp.py [--seconds 20] [--idle 2]
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
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--idle", type=float, default=2.0)
    ap.add_argument("--params", type=int, default=25_600_000)
    args = ap.parse_args()
    pkg = importlib.import_module(PKG)
    np.random.seed(1234)
    T = 200_000
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, 8, T, True)
    g = pkg.VirtualWorkerGroup(GP, numel=args.params)
    for r in range(8):
        pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[r].data_ptr(), args.params, 1234 + r, None))
    torch.cuda.synchronize()
    time.sleep(args.idle)
    B = 100
    blocks = []
    it = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(B):
            g.step(it % T)
            it += 1
        b.record()
        b.synchronize()
        blocks.append((time.perf_counter() - t0, 1e3 * a.elapsed_time(b) / B))
    us = np.array([x[1] for x in blocks])
    out = {"rounds": it, "block": B, "first_blocks_us": [round(x, 1) for x in us[:10]],
           "by_second": {}, "min_us": float(us.min()), "last_10_mean_us": float(us[-10:].mean())}
    for s in range(int(args.seconds) + 1):
        sel = [u for t, u in blocks if s <= t < s + 1]
        if sel:
            out["by_second"][s] = round(float(np.mean(sel)), 1)
    out["frac_last_10"] = 2 * 8 * args.params * 4 / (out["last_10_mean_us"] * 1e-6) / 8e12
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
