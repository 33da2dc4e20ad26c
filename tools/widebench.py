"""Throughput of the mixing kernels by slot count on one GPU: ER topologies decomposed by the host
path, full rounds, arena of about 1.6 GB of rows; HBM GB/s on the algorithmic bytes (2 x rows x P x 4)."""
import importlib
import json
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
from conftest import Topo  # noqa: E402

ROW_BYTES = int(float(os.environ.get("WIDE_BYTES", 1.6384e9)))
CASES = [(64, 0.1), (96, 0.06), (128, 0.05), (150, 0.04), (48, 0.9)]
if os.environ.get("WIDE_CASES"):                 # e.g. WIDE_CASES=96:0.06,150:0.04
    CASES = [(int(a), float(b)) for a, b in (c.split(":") for c in os.environ["WIDE_CASES"].split(","))]
# WIDE_TUNE=wide_lds_kb=80 (one setting) or WIDE_SWEEP="wide_lds_kb=40;wide_lds_kb=80,wide_per_cu=2"
SWEEP = os.environ.get("WIDE_SWEEP", os.environ.get("WIDE_TUNE", "")).split(";")
DEFAULT = pkg.engine.mix_tuning()


def run(n, p, tune):
    random.seed(0)
    gp = pkg.GraphProcessor(pkg.erdos_renyi(n, p, 1234), 1.0, 0, n, 4, False)
    M = len(gp.neighbors_info)
    P = ROW_BYTES // (2 * 4 * n) // 256 * 256
    topo = Topo(gp.neighbors_info, 0.5 / M, np.ones((64, M), np.uint8))
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    for i in range(n):
        pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 7 + i, None)
    for j in range(5):
        grp.step(j)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for j, (a, b) in enumerate(ev):
        a.record()
        grp.step(5 + j)
        b.record()
    torch.cuda.synchronize()
    us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
    byts = 2 * n * P * 4
    print(json.dumps({"tune": tune, "workers": n, "matchings": M, "slots": grp.engine.n_slots,
                      "kernel": "mix_kernel_wide" if (n > 64 or M > 32) else pkg.engine.mix_kernel_name(n),
                      "P": P, "us": round(us, 1), "TBps": round(byts / us / 1e6, 3)}), flush=True)
    del grp
    torch.cuda.empty_cache()


for tune in SWEEP:
    pkg.engine.set_mix_tuning(**DEFAULT)
    if tune:
        pkg.engine.set_mix_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in tune.split(","))})
    for n, p in CASES:
        run(n, p, tune)
