"""Host cost of one eager gossip round (the launch-bound configs' host-clocked figures): wall time
per call over 20,000 back-to-back calls of each layer of the path -- VirtualWorkerGroup.step,
GossipEngine.mix, the ctypes call of mx_gossip_mix with prebuilt arguments -- on a tiny row
(P = 256: the kernel finishes before the host issues the next, so the wall time is the host's),
beside torch's own launch of a one-element add_ for scale.  One JSON line.

    python tools/launch_overhead.py
"""
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


def per_call_us(fn, n=20_000):
    for i in range(200):
        fn(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(n):
        fn(i)
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t) / n


def main():
    pkg = importlib.import_module(PKG)
    np.random.seed(1234)
    T = 1000
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, 8, T, True)
    g = pkg.VirtualWorkerGroup(GP, numel=256)
    eng, lay, L = g.engine, g.layout, pkg.lib
    sp = pkg._lib.stream_ptr
    args = lay._args + (eng._plan_ptr,)
    x = torch.zeros(1, device="cuda")
    out = {
        "step_us": per_call_us(lambda i: g.step(i % T)),
        "engine_mix_us": per_call_us(lambda i: eng.mix(i % T, lay)),
        "ctypes_mix_us": per_call_us(lambda i: L.mx_gossip_mix(*args, i % T, eng.n_local, eng.M, eng.alpha32, sp())),
        "torch_add_us": per_call_us(lambda i: x.add_(1.0)),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
