"""One rank of the pull-transport stress test (tests/test_gpu_multiproc.py launches 4 via torchrun,
all sharing GPU 0).  Rounds are enqueued back to back with no host synchronisation, but every rank
sleeps a random 0-3 ms before some of its rounds, so the ranks drift several rounds apart and the
device gates really wait: a rank that runs ahead must be held at its gate until the partners it
reads have published, and must not overwrite a snapshot a slower partner is still reading.  Whole
rows (decen) and Choco messages (fetch and direct reads), every worker vs the oracle at the end.
Exit status 0 = all matched."""
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
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)
import oracle as O  # noqa: E402
from conftest import PKG_NAME, Topo, pull_clean, report_rank_errors  # noqa: E402
from gloo_transport import gather_rows  # noqa: E402
from mp_worker import by_worker  # noqa: E402


def topo_of(pkg, gid, rounds, seed, alpha):
    n = pkg.GRAPH_SIZES[gid]
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    flags = (np.random.RandomState(seed).uniform(size=(rounds, M)) < 0.7).astype(np.uint8)
    flags[0] = 1
    return n, Topo(gp.neighbors_info, alpha, flags), flags


def jitter(rng):
    if rng.uniform() < 0.4:
        time.sleep(rng.uniform(0, 3e-3))


def decen(pkg, rank, world, rounds=60, P=50_021):
    n, topo, flags = topo_of(pkg, 2, rounds, 31, 0.17)
    grp = pkg.VirtualWorkerGroup(topo, numel=P, rank=rank, nranks=world, comm=pkg.PullTransport(timeout_s=60),
                                 placement="auto")
    X = np.stack([O.synth(300 + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X[grp.workers]))
    torch.cuda.synchronize()
    rng = np.random.RandomState(1000 + rank)
    for it in range(rounds):
        jitter(rng)
        grp.step(it)
        if flags[it].any():
            X = O.decen_round(X, topo.neighbors_info, flags[it], 0.17)
    grp.wait_round()
    got = by_worker(grp, gather_rows(grp.rows, grp.row_base, n))
    rounds_run = grp._pull.round
    grp.close()
    return bool(np.array_equal(got.view(np.uint32), X.view(np.uint32))) and rounds_run >= rounds // 2


def choco(pkg, rank, world, pull_read, rounds=40, P=40_009):
    n, topo, flags = topo_of(pkg, 0, rounds, 37, 2 / 7)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=0.95, consensus_lr=0.2, rank=rank, nranks=world,
                               comm=pkg.PullTransport(timeout_s=60), placement="auto", pull_read=pull_read)
    X = np.stack([O.synth(400 + i, P) for i in range(n)])
    XH = np.zeros_like(X)
    S = np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X[grp.workers]))
    torch.cuda.synchronize()
    rng = np.random.RandomState(2000 + rank)
    partner = np.asarray(topo.neighbors_info, np.int32)
    for it in range(rounds):
        jitter(rng)
        grp.step(it)
        if flags[it].any():
            O.choco_round(X, XH, S, partner, flags[it], 2 / 7, grp.k, 0.2)
    grp.wait_round()
    grp.check_topk()
    got = [by_worker(grp, gather_rows(t[:, :P], grp.row_base, n)) for t in (grp.x, grp.x_hat, grp.s)]
    grp.close()
    return all(bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))) for a, b in zip(got, (X, XH, S)))


def main():
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    rank, world = dist.get_rank(), dist.get_world_size()
    pkg = importlib.import_module(PKG_NAME)
    res = {"decen_g2": decen(pkg, rank, world),
           "choco_fetch": choco(pkg, rank, world, "fetch"),
           "choco_direct": choco(pkg, rank, world, "direct")}
    res["pull_ipc_clean"] = pull_clean(pkg, min_binds=3)
    torch.cuda.synchronize()
    flags = [None] * world
    dist.all_gather_object(flags, all(res.values()))
    if rank == 0:
        print(json.dumps({"world": world, "all_ranks": all(flags), **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if all(flags) else 1)


if __name__ == "__main__":
    report_rank_errors(main)
