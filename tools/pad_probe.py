"""Row-stride probe: the headline mixing round (graph 0, 8 x 25.6M fp32, full round) with the arena
rows padded by `pad` extra floats (the kernel mixes them too: <= 0.3 % more bytes), alternating
pads twice, against torch copy_ of the same bytes in the same run.  Tests whether the 8 concurrent
row streams' relative placement (HBM channel / bank mapping) is what makes some boxes slower."""
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


def timeit(fn, reps=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


P = 25_600_000
gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
topo = Topo(gp.neighbors_info, 2 / 7, np.ones((4, len(gp.neighbors_info)), np.uint8))
pads = [int(x) for x in os.environ.get("PADS", "0,64,1024,4096,16448,65600,262208").split(",")]
for rep in range(2):
    for pad in pads:
        grp = pkg.VirtualWorkerGroup(topo, numel=P + pad)
        for i in range(8):
            pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P + pad, 1234 + i, None)
        ms = timeit(lambda: grp.engine.mix(0, grp.layout))
        byts = 2 * 8 * (P + pad) * 4
        print(json.dumps({"rep": rep, "pad": pad, "ld": grp.ld, "us": round(ms * 1e3, 1),
                          "TBps": round(byts / ms / 1e9, 3)}), flush=True)
        del grp
        torch.cuda.empty_cache()
src = torch.empty(8 * P, device="cuda")
dst = torch.empty_like(src)
ms = timeit(lambda: dst.copy_(src))
print(json.dumps({"torch_copy_us": round(ms * 1e3, 1)}), flush=True)
