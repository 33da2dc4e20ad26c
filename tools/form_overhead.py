"""Fixed per-round cost of each N > 1 exchange form, one torchrun rank per process.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/form_overhead.py [P] [K]

Graph 0, 8 workers in contiguous blocks, every matching active every round, P floats per worker
(default 100,000: the mixing kernel itself is a few microseconds, so ms/round is the form's fixed
cost).  Per form: 5 untimed rounds, then K rounds back to back between synchronize + barrier on
both sides, max over ranks.  Forms:
  plain    -- exchange through the gloo test transport (tests/gloo_transport.py), then the mix:
              RCCL's stand-in on a one-GPU box (RCCL refuses two ranks on one device)
  chunked  -- the same, column-pipelined in 4 chunks on a side stream
  pull     -- PullTransport (IPC-mapped snapshots read by the mixing kernel)
  mix_only -- the pull group's mixing launches alone (no publish, gate or exchange)
and the same for ChocoSGD rounds (top-1 %, same P): choco_plain (messages over the gloo stand-in),
choco_pull (the apply reads them from the owners' snapshots behind the device gate) and choco_null
(a transport that moves nothing: compress + apply alone).
Prints one JSON line (rank 0)."""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from conftest import PKG_NAME, Topo  # noqa: E402
from gloo_transport import GlooTransport  # noqa: E402


def timed(world, fn, first, K):
    torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter()
    for j in range(K):
        fn(first + j)
    torch.cuda.synchronize()
    dist.barrier()
    el = torch.tensor([time.perf_counter() - t])
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return 1e3 * float(el) / K


def main():
    import importlib
    P = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    pkg = importlib.import_module(PKG_NAME)
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
    T = 5 + 3 * K + 8
    topo = Topo(gp.neighbors_info, 2 / 7, np.ones((T, len(gp.neighbors_info)), np.uint8))
    res = {"world": world, "P": P, "K": K}
    forms = {"plain": dict(comm=GlooTransport(pkg)),
             "chunked": dict(comm=GlooTransport(pkg), chunk_cols=(P + 3) // 4),
             "pull": dict(comm=pkg.PullTransport())}
    for name, kw in forms.items():
        g = pkg.VirtualWorkerGroup(topo, numel=P, rank=rank, nranks=world, **kw)
        for it in range(5):
            g.step(it)
        res[name + "_ms"] = timed(world, g.step, 5, K)
        if name == "pull":
            res["mix_only_ms"] = timed(world, lambda it: g.engine.mix(it, g.layout), 5 + K, K)
            st = g._pull
            res["pull_rounds"] = int(st.round)
        g.close()
    class NullComm:
        handle = None

        def __init__(self):
            self.rank, self.nranks = rank, world

        def exchange_round(self, *a):
            return 0

    cforms = {"choco_plain": GlooTransport(pkg), "choco_pull": pkg.PullTransport(), "choco_null": NullComm()}
    for name, comm in cforms.items():
        g = pkg.ChocoWorkerGroup(topo, numel=P, ratio=0.99, consensus_lr=0.1, rank=rank, nranks=world, comm=comm)
        for r in range(g.n_local):
            pkg._lib.check(pkg.lib.mx_synth_fill(g.rows[r].data_ptr(), P, 1234 + g.workers[r], None))
        for it in range(5):
            g.step(it)
        res[name + "_ms"] = timed(world, g.step, 5, K)
        if name == "choco_pull":
            res["choco_pull_rounds"] = int(g._pull.round)
        g.close()
    if rank == 0:
        for name in forms:
            res[name + "_overhead_ms"] = res[name + "_ms"] - res["mix_only_ms"]
        for name in ("choco_plain", "choco_pull"):
            res[name + "_overhead_ms"] = res[name + "_ms"] - res["choco_null_ms"]
        print(json.dumps(res), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
