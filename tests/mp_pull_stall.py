"""Two ranks sharing GPU 0 under PullTransport; rank 1 stalls before its third round (launched by
tests/test_gpu_multiproc.py via torchrun).

Rank 0's third round enqueues its snapshot and the gate, whose bounded wait for rank 1's epoch
expires after the transport's 2 s deadline: communicate() must raise MXError naming rank 1 instead
of hanging.  Rank 1 then wakes up and runs its third round, which completes (rank 0 published its
epoch before waiting).  Rank 0 prints one JSON line."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)
from conftest import PKG_NAME, Topo, pull_clean, report_rank_errors  # noqa: E402

TIMEOUT_S = 2.0


def main():
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    pkg = importlib.import_module(PKG_NAME)
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, 8, 4, True)
    topo = Topo(gp.neighbors_info, 2 / 7, np.ones((8, len(gp.neighbors_info)), np.uint8))
    grp = pkg.VirtualWorkerGroup(topo, numel=20_000, rank=rank, nranks=2,
                                 comm=pkg.PullTransport(timeout_s=TIMEOUT_S))
    res = {"first_rounds_ok": True, "raised": False, "message": None, "seconds": None}
    for _ in range(2):
        grp.communicate()
    if rank == 1:
        time.sleep(3 * TIMEOUT_S)
        grp.communicate()                          # rank 0's epoch 3 is out: completes
        res["peer_round_ok"] = True
    else:
        t = time.perf_counter()
        try:
            grp.communicate()
        except pkg.MXError as e:
            res["raised"], res["message"] = True, str(e)
        res["seconds"] = time.perf_counter() - t
        try:                                        # sticky: the next round raises at once
            grp.step(3)
            res["sticky"] = False
        except pkg.MXError:
            res["sticky"] = True
    res["pull_ipc_clean"] = pull_clean(pkg, min_binds=1)
    objs = [None, None]
    dist.all_gather_object(objs, res)
    grp._pull.close()                               # the ranks met above; nothing reads any more
    grp._pull = None
    if rank == 0:
        out = dict(objs[0])
        out["peer_round_ok"] = bool(objs[1].get("peer_round_ok"))
        out["pull_ipc_clean"] = all(o["pull_ipc_clean"] for o in objs)
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    report_rank_errors(main)
