"""Per-GPU compute of the N > 1 layouts, measured on one GPU: for N = 2 / 4 / 8 every rank's
share (placement "auto", as bench.py) is built with a null transport (the exchange is skipped;
slab rows / received messages hold valid stand-in data), and the mixing kernel (decen, 8 x 25.6M)
and the Choco round (VGG-16 size, ratio 0.99) are timed per rank with HIP events.  The maximum
over ranks is what each GPU adds to the RCCL exchange in a real N-GPU round."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")


class NullComm:
    """Skips the transfer; reports the receive count the native exchange plan would post."""

    def __init__(self, rank, nranks):
        self.rank, self.nranks, self.handle = rank, nranks, None

    def exchange_round(self, engine, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes):
        return int(sum(1 for op in engine.exchange_plan(it) if op[0] == 1))


def ev_time(fn, reps):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for j, (a, b) in enumerate(ev):
        a.record()
        fn(j + 3)
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


n = 8
P = int(os.environ.get("PERGPU_P", 25_600_000))
PC = int(os.environ.get("PERGPU_CHOCO_P", 14_774_436))
T = 40
np.random.seed(1234)
GP = pkg.MatchaProcessor(pkg.select_graph(0), 1.0, 0, n, T, True)
for N in [int(x) for x in os.environ.get("PERGPU_NS", "1,2,4,8").split(",")]:
    mix_ms, choco_ms, slots = [], [], []
    for r in range(N):
        comm = NullComm(r, N) if N > 1 else None
        g = pkg.VirtualWorkerGroup(GP, numel=P, rank=r, nranks=N, comm=comm, placement="auto" if N > 1 else None)
        for i in range(g.n_local):
            pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[i].data_ptr(), P, 1234 + g.workers[i], None))
        if g.slab is not None:
            g.slab.zero_()
        mix_ms.append(ev_time(lambda it: g.engine.mix(it, g.layout), 20) if not os.environ.get("PERGPU_NO_MIX") else 0.0)
        slots.append(g.engine.n_slots)
        del g
        torch.cuda.empty_cache()
        c = pkg.ChocoWorkerGroup(GP, numel=PC, ratio=0.99, consensus_lr=0.1, rank=r, nranks=N, comm=comm,
                                 placement="auto" if N > 1 else None)
        for i in range(c.n_local):
            pkg._lib.check(pkg.lib.mx_synth_fill(c.rows[i].data_ptr(), PC, 1234 + c.workers[i], None))
        c.compress(0)
        torch.cuda.synchronize()
        for s in range(c.n_local, c.engine.n_slots):       # received messages: valid stand-ins
            c.msgs[s * c.msg_ld:(s + 1) * c.msg_ld].copy_(c.msgs[:c.msg_ld])
        sweep = os.environ.get("PERGPU_TOPK_SWEEP")     # e.g. "compact_blocks=1024,2048;sample_pieces=1,4"
        if sweep:
            import itertools
            axes = [(kv.split("=")[0], [int(v) for v in kv.split("=")[1].split(",")]) for kv in sweep.split(";")]
            saved = {k: int(pkg.lib.mx_topk_get(k.encode())) for k, _ in axes}
            for combo in itertools.product(*[v for _, v in axes]):
                for (k, _), v in zip(axes, combo):
                    pkg._lib.check(pkg.lib.mx_topk_set(k.encode(), v))
                ms = ev_time(lambda it: c.step(it), 10)
                print(json.dumps({"gpus": N, "rank": r, "n_local": c.n_local,
                                  **{k: v for (k, _), v in zip(axes, combo)}, "choco_ms": round(ms, 4)}), flush=True)
            for k, v in saved.items():
                pkg._lib.check(pkg.lib.mx_topk_set(k.encode(), v))
        choco_ms.append(ev_time(lambda it: c.step(it), 10))
        del c
        torch.cuda.empty_cache()
    print(json.dumps({"gpus": N, "slots_per_rank": slots, "mix_ms_per_rank": [round(x, 4) for x in mix_ms],
                      "mix_ms_max": round(max(mix_ms), 4), "choco_ms_per_rank": [round(x, 4) for x in choco_ms],
                      "choco_ms_max": round(max(choco_ms), 4)}), flush=True)
