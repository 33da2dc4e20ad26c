"""Same-box A/B of the host-model staging path: the round-1 _Staging (one torch.cat into a pinned
buffer + one DMA each way, a device sync before the scatter back) vs the current one (16 MB
pieces, each piece's DMA issued as soon as it is filled / scattered as soon as it arrives).
8 host models x 25.6M fp32 in 54 tensors, as bench.py's staged figure."""
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
pkg = importlib.import_module(PKG)
C = importlib.import_module(PKG + ".communicator")


class OldStaging(C._Staging):
    def load(self):
        pin = self._pinned()
        torch.cat([p.data.reshape(-1) for p in self.params], out=pin)
        self.row.copy_(pin, non_blocking=True)

    def store(self):
        pin = self._pinned()
        pin.copy_(self.row, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        with torch.no_grad():
            for f, t in zip(pkg.unflatten_tensors(pin, [p.data for p in self.params]), self.params):
                t.data.copy_(f)


P, n, K = int(os.environ.get("STAGE_P", 25_600_000)), 8, 3
GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, n, 40, True)
grp = pkg.VirtualWorkerGroup(GP, numel=P)
cuts = np.linspace(0, P, 55).astype(np.int64)
models = []
for r in range(n):
    pkg._lib.check(pkg.lib.mx_synth_fill(grp.rows[r].data_ptr(), P, 1234 + r, None))
    row = grp.rows[r].cpu()
    models.append([torch.nn.Parameter(row[a:b].clone()) for a, b in zip(cuts[:-1], cuts[1:])])
res = {"old": [], "new": []}
it = 0
for rep in range(3):
    for name, cls in (("old", OldStaging), ("new", C._Staging)):
        st = [cls(ps, grp.rows[r]) for r, ps in enumerate(models)]
        for s in st:                     # warm: pinned buffers, plans
            s.load()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for j in range(K):
            for s in st:
                s.load()
            grp.step(it)
            it += 1
            torch.cuda.synchronize()
            for s in st:
                s.store()
        res[name].append(1e3 * (time.perf_counter() - t) / K)
        del st
print(json.dumps({k: [round(x, 2) for x in v] for k, v in res.items()}))
