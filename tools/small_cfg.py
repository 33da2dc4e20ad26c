"""Config 2 (CIFAR ResNet(18,100), 181,668 params x 8 workers, MATCHA C_b = 0.5, graph 0) and
config 1 (MLP, 666,547 params) rounds on one GPU: eager and HIP-graph-replayed rounds/s, for
kernel traces of the launch-bound small rows (run under rocprofv3 --kernel-trace --stats).
SMALL_TUNE="key=value,..." applies mix tuning first; SMALL_K rounds per timing (default 200)."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")

K = int(os.environ.get("SMALL_K", 200))
W = 5
DEFAULT = pkg.engine.mix_tuning()
for tune in os.environ.get("SMALL_TUNE", "").split(";"):
    pkg.engine.set_mix_tuning(**DEFAULT)
    if tune:
        pkg.engine.set_mix_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in tune.split(","))})
    cases = (("resnet18_100_matcha0.5", 181_668, 0.5), ("mlp_matcha0.5", 666_547, 0.5),
             ("resnet18_100_full", 181_668, 1.0))
    if os.environ.get("SMALL_P"):                # e.g. SMALL_P=1000000,2000000 (MATCHA 0.5 rows of that size)
        cases = tuple((f"P{p}_matcha0.5", int(float(p)), 0.5) for p in os.environ["SMALL_P"].split(","))
    for name, P, budget in cases:
        np.random.seed(1234)
        gp = pkg.MatchaProcessor(pkg.select_graph(0), budget, 0, 8, 2 * (W + K) + 2, True)
        g = pkg.VirtualWorkerGroup(gp, numel=P)
        for i in range(8):
            pkg.lib.mx_synth_fill(g.rows[i].data_ptr(), P, 7 + i, None)
        for it in range(W):
            g.step(it)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for it in range(W, W + K):
            g.step(it)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t) / K
        gr = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            with torch.cuda.graph(gr):
                g.device_rounds(K)
        torch.cuda.synchronize()
        g.iter_dev.fill_(W)
        gr.replay()
        g.iter_dev.fill_(W)
        torch.cuda.synchronize()
        t = time.perf_counter()
        gr.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t) / K
        print(json.dumps({"tune": tune, "config": name, "P": P, "kernel": pkg.engine.mix_kernel_name(8),
                          "eager_us": round(eager * 1e6, 2), "graph_us": round(graph * 1e6, 2)}), flush=True)
        del gr
        g.close()
        del g
        torch.cuda.empty_cache()
