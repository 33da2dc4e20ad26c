"""One rank of the multi-process GPU test (launched by tests/test_gpu_multiproc.py via torchrun).

Every rank shares GPU 0 and holds a contiguous block of the topology's workers; partner rows
cross process boundaries through tests/gloo_transport.GlooTransport (RCCL refuses two ranks on
one GPU).  Each case runs several rounds, gathers all rows and compares them bit-exactly with the
single-process oracle.  Exit status 0 = every case matched."""
import importlib
import json
import os
import sys

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
from gloo_transport import GlooTransport, gather_rows  # noqa: E402
from reforder import mpi4py_sum as _mpi4py_sum  # noqa: E402


def by_worker(grp, rows):
    """gathered rows are in the group's position order; put them in worker order"""
    if grp.placement is None:
        return rows
    out = np.empty_like(rows)
    out[grp.placement] = rows
    return out


def decen_case(pkg, T, gid, P, rounds, chunk_cols=None, seed=5, placement=None, back_to_back=False):
    """rounds through communicate() (a wait per round), or with back_to_back all rounds enqueued
    by step() with no host wait between them (one synchronize at the end)"""
    rank, world = dist.get_rank(), dist.get_world_size()
    n = pkg.GRAPH_SIZES[gid]
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    rng = np.random.RandomState(seed)
    flags = (rng.uniform(size=(rounds, M)) < 0.6).astype(np.uint8)
    flags[0] = 1
    topo = Topo(gp.neighbors_info, 0.21, flags)
    grp = pkg.VirtualWorkerGroup(topo, numel=P, rank=rank, nranks=world, comm=T, chunk_cols=chunk_cols,
                                 placement=placement)
    X = np.stack([O.synth(77 + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X[grp.workers]))
    for it in range(rounds):
        if back_to_back:
            grp.step(it)
        else:
            grp.communicate()
        if flags[it].any():
            X = O.decen_round(X, topo.neighbors_info, flags[it], 0.21)
    if back_to_back:
        grp.wait_round()
    got = by_worker(grp, gather_rows(grp.rows, grp.row_base, n))
    grp.close()
    return bool(np.array_equal(got.view(np.uint32), X.view(np.uint32)))


def pull_rows_case(pkg, gid, P, rounds, seed=21, placement=None):
    """The reference's averaging(active_flags) with arbitrary rows under the pull transport: each
    round's row is drawn at random (the same on every rank), its plan record found or built by
    engine.record_for (a schedule iteration with the same row, else the scratch record -- then the
    gate reads the scratch row), and the rounds enqueued back to back with no host wait; every
    worker's row vs the oracle at the end."""
    rank, world = dist.get_rank(), dist.get_world_size()
    n = pkg.GRAPH_SIZES[gid]
    gp = pkg.GraphProcessor(pkg.select_graph(gid), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    sched = np.zeros((3, M), np.uint8)
    sched[0] = 1
    sched[1, ::2] = 1
    topo = Topo(gp.neighbors_info, 0.19, sched)
    grp = pkg.VirtualWorkerGroup(topo, numel=P, rank=rank, nranks=world, comm=pkg.PullTransport(), placement=placement)
    X = np.stack([O.synth(500 + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X[grp.workers]))
    rng = np.random.RandomState(seed)
    adhoc = 0
    for _ in range(rounds):
        f = (rng.uniform(size=M) < 0.5).astype(np.uint8)
        if rng.uniform() < 0.3:
            f = sched[rng.randint(2)].copy()
        it = grp.engine.record_for(f)
        adhoc += it == grp.engine.T
        if f.any():
            grp.step(it)
            X = O.decen_round(X, topo.neighbors_info, f, 0.19)
    grp.wait_round()
    got = by_worker(grp, gather_rows(grp.rows, grp.row_base, n))
    grp.close()
    return bool(np.array_equal(got.view(np.uint32), X.view(np.uint32))) and adhoc > 0


def choco_case(pkg, T, P, ratio, rounds, seed=9, placement=None, back_to_back=False, pull_read="fetch"):
    """x and x_hat of every worker vs the oracle's Choco rounds; with back_to_back all rounds are
    enqueued by step() with no host wait between them (the pull transport's device gate alone
    orders them across ranks)"""
    rank, world = dist.get_rank(), dist.get_world_size()
    n = 8
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    rng = np.random.RandomState(seed)
    flags = (rng.uniform(size=(rounds, M)) < 0.6).astype(np.uint8)
    flags[0] = 1
    topo = Topo(gp.neighbors_info, 2 / 7, flags)
    kw = {"pull_read": pull_read} if isinstance(T, pkg.PullTransport) else {}
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=ratio, consensus_lr=0.1, rank=rank, nranks=world, comm=T,
                               placement=placement, **kw)
    X = np.stack([O.synth(99 + i, P) for i in range(n)])
    XH = np.zeros_like(X)
    S = np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X[grp.workers]))
    for it in range(rounds):
        if back_to_back:
            grp.step(it)
        else:
            grp.communicate()
        if flags[it].any():
            O.choco_round(X, XH, S, np.asarray(topo.neighbors_info, np.int32), flags[it], 2 / 7, grp.k, 0.1)
    if back_to_back:
        grp.wait_round()
        grp.check_topk()
    got = by_worker(grp, gather_rows(grp.rows, grp.row_base, n))
    gxh = by_worker(grp, gather_rows(grp.x_hat[:, :P], grp.row_base, n))
    gs = by_worker(grp, gather_rows(grp.s[:, :P], grp.row_base, n))
    grp.close()
    return bool(np.array_equal(got.view(np.uint32), X.view(np.uint32)) and
                np.array_equal(gxh.view(np.uint32), XH.view(np.uint32)) and
                np.array_equal(gs.view(np.uint32), S.view(np.uint32)))


def choco_pull_rows_case(pkg, P, rounds, seed=23, placement=None):
    """ChocoCommunicator.averaging(active_flags) with arbitrary rows under the pull transport: a
    random row per round (the same on every rank), its plan record found or built by
    engine.record_for, rounds enqueued back to back (compress + publish + gate + apply) with no
    host wait; x / x_hat / s of every worker vs the oracle at the end."""
    rank, world = dist.get_rank(), dist.get_world_size()
    n = 8
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    M = len(gp.neighbors_info)
    sched = np.zeros((3, M), np.uint8)
    sched[0] = 1
    sched[1, ::2] = 1
    topo = Topo(gp.neighbors_info, 2 / 7, sched)
    grp = pkg.ChocoWorkerGroup(topo, numel=P, ratio=0.95, consensus_lr=0.15, rank=rank, nranks=world,
                               comm=pkg.PullTransport(), placement=placement)
    X = np.stack([O.synth(700 + i, P) for i in range(n)])
    XH = np.zeros_like(X)
    S = np.zeros_like(X)
    grp.rows.copy_(torch.from_numpy(X[grp.workers]))
    rng = np.random.RandomState(seed)
    partner = np.asarray(topo.neighbors_info, np.int32)
    adhoc = 0
    for _ in range(rounds):
        f = (rng.uniform(size=M) < 0.5).astype(np.uint8)
        if rng.uniform() < 0.3:
            f = sched[rng.randint(2)].copy()
        it = grp.engine.record_for(f)
        adhoc += it == grp.engine.T
        if f.any():
            grp.step(it)
            O.choco_round(X, XH, S, partner, f, 2 / 7, grp.k, 0.15)
    grp.wait_round()
    grp.check_topk()
    got = [by_worker(grp, gather_rows(t[:, :P], grp.row_base, n)) for t in (grp.x, grp.x_hat, grp.s)]
    grp.close()
    return all(bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))) for a, b in zip(got, (X, XH, S))) \
        and adhoc > 0


def centralized_case(pkg, T):
    """centralizedCommunicator through the product path (gather over the transport, then the
    native mx_mean_rows in the reference's order + the div_ of communicator.py:62) on random rows:
    bit-exact for "tree" / "sequential", within 1e-6 relative for "ring"."""
    rank, world = dist.get_rank(), dist.get_world_size()
    ok = True
    for order in ("tree", "sequential", "ring"):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.Linear(200, 77)).cuda()
        shapes = [p.shape for p in m.parameters()]
        P = sum(p.numel() for p in m.parameters())
        rows = [O.synth(555 + r, P) * np.float32(10.0 ** (r % 3)) for r in range(world)]
        with torch.no_grad():
            off = 0
            for p in m.parameters():
                p.copy_(torch.from_numpy(rows[rank][off:off + p.numel()].reshape(p.shape)))
                off += p.numel()
        pkg.centralizedCommunicator(rank, world, transport=T, order=order).communicate(m)
        got = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy()
        assert [p.shape for p in m.parameters()] == shapes
        if order == "ring":
            want = _mpi4py_sum(rows, "tree") / np.float32(world)
            scale = np.abs(np.stack(rows)).sum(0) / np.float32(world)   # reassociation bound
            ok &= bool(np.all(np.abs(got - want) <= 1e-6 * scale))
        else:
            want = _mpi4py_sum(rows, order) / np.float32(world)
            ok &= bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    return ok


def main():
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    pkg = importlib.import_module(PKG_NAME)
    T = GlooTransport(pkg)
    res = {
        "decen_g0": decen_case(pkg, T, 0, 30_011, 5),
        "decen_g2": decen_case(pkg, T, 2, 9_001, 4),
        "decen_g0_chunked": decen_case(pkg, T, 0, 70_001, 4, chunk_cols=16_384),
        "choco_g0": choco_case(pkg, T, 40_003, 0.9, 4),
        "decen_g2_placed": decen_case(pkg, T, 2, 9_001, 4, placement="auto"),
        "choco_g0_placed": choco_case(pkg, T, 20_011, 0.9, 3, placement="auto"),
        "centralized": centralized_case(pkg, T),
        # the pull transport: peers map each rank's IPC-shared snapshot buffer and the mixing
        # kernel reads partner rows from it (processes share GPU 0 here; xGMI on a real node)
        "decen_g0_pull": decen_case(pkg, pkg.PullTransport(), 0, 30_011, 6),
        "decen_g2_pull_placed": decen_case(pkg, pkg.PullTransport(), 2, 9_001, 5, placement="auto"),
        # 40 device-gated rounds (no host barrier per round): each snapshot buffer reused 20 times
        "decen_g0_pull_long": decen_case(pkg, pkg.PullTransport(), 0, 30_011, 40, seed=11, back_to_back=True),
        "decen_g2_pull_rows_placed": pull_rows_case(pkg, 2, 12_007, 24, placement="auto"),
        # Choco under the pull transport: the partners' top-k messages read by the apply pass from
        # the owners' snapshot buffers (each reused 3 / 7 times), communicate() and back to back
        "choco_g0_pull": choco_case(pkg, pkg.PullTransport(), 40_003, 0.9, 6),
        "choco_g0_pull_long_placed": choco_case(pkg, pkg.PullTransport(), 20_011, 0.9, 14, seed=13,
                                                placement="auto", back_to_back=True),
        "choco_g0_pull_rows_placed": choco_pull_rows_case(pkg, 15_013, 16, placement="auto"),
        "choco_g0_pull_direct_long_placed": choco_case(pkg, pkg.PullTransport(), 20_011, 0.9, 14, seed=17,
                                                       placement="auto", back_to_back=True, pull_read="direct"),
        # edge shapes under pull: one entry per message (k = 1, the reference's argmax branch) on a
        # row shorter than one 4096-element tile, and an odd k on a ragged last tile
        "choco_g0_pull_k1": choco_case(pkg, pkg.PullTransport(), 1_000, 0.9995, 5, seed=3, back_to_back=True),
        "choco_g0_pull_odd_k": choco_case(pkg, pkg.PullTransport(), 12_389, 0.99, 5, seed=4),
    }
    res["pull_ipc_clean"] = pull_clean(pkg, min_binds=8)     # no refused export, no failed bind
    torch.cuda.synchronize()
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if all(res.values()) else 1)


if __name__ == "__main__":
    report_rank_errors(main)
