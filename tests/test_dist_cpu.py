"""Multi-rank exchange contract on CPU (gloo, world_size 2, 4 and 8 -- the driver's 8-GPU layout).

Each rank holds a contiguous block of the 8 workers of graph 0.  Per round it posts, in the
order mx_exchange_plan (the native enumeration mx_exchange_round feeds to RCCL) returns, a
gloo isend of every local row whose partner is remote and an irecv of every remote partner row
into its receive slab.  Checks: every slab slot holds exactly the row the round plan expects
there (tests/planref.py, itself pinned to the GPU plan kernel in test_gpu_gossip.py), and the
per-rank FMA-chain result assembled from local rows + slab equals the single-process oracle.
"""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exchange_plan(lib, flags_row, partner, owner, rank, row_base, n_local):
    M, n = partner.shape
    fr = np.ascontiguousarray(flags_row, np.uint8)
    cnt = ctypes.c_int(0)
    assert lib.mx_exchange_plan(fr.ctypes.data, M, partner.ctypes.data, n, owner.ctypes.data, rank,
                                row_base, n_local, None, 0, ctypes.byref(cnt)) == 0
    ops = np.zeros((max(1, cnt.value), 4), np.int32)
    assert lib.mx_exchange_plan(fr.ctypes.data, M, partner.ctypes.data, n, owner.ctypes.data, rank,
                                row_base, n_local, ops.ctypes.data, cnt.value, ctypes.byref(cnt)) == 0
    return ops[:cnt.value]


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, HERE)
        import torch
        import torch.distributed as dist
        from conftest import PKG_NAME  # noqa: F401
        import importlib
        import oracle as O
        from planref import py_plan
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        pkg = importlib.import_module(PKG_NAME)
        lib = pkg.lib
        n, P, alpha = 8, 1003, 2 / 7
        gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
        partner = np.ascontiguousarray(np.asarray(gp.neighbors_info, np.int32))
        M = partner.shape[0]
        owner = pkg.engine.owner_table(n, world)
        row_base, n_local = pkg.partition(n, world)[rank]
        X = np.stack([O.synth(77 + i, P) for i in range(n)])          # global truth
        rng = np.random.RandomState(5)
        flags = (rng.uniform(size=(12, M)) < 0.6).astype(np.uint8)
        flags[0] = 1
        for f in flags:
            ops = _exchange_plan(lib, f, partner, owner, rank, row_base, n_local)
            any_, nrem, src, sw, senders = py_plan(f, partner, row_base, n_local, alpha)
            slab = torch.zeros((max(1, nrem), P))
            local = torch.from_numpy(X[row_base:row_base + n_local].copy())
            reqs = []
            for kind, peer, idx, who in ops:
                if kind == 0:
                    assert who == row_base + idx
                    reqs.append(dist.isend(local[idx].contiguous(), dst=int(peer)))
                else:
                    assert senders[idx] == who and owner[who] == peer
                    reqs.append(dist.irecv(slab[idx], src=int(peer)))
            for r in reqs:
                r.wait()
            assert sum(1 for o in ops if o[0] == 1) == nrem
            for k in range(nrem):
                assert np.array_equal(slab[k].numpy(), X[senders[k]]), "slab slot holds the wrong row"
            # every local row's partner walk resolves to the right workers
            for r in range(n_local):
                w = row_base + r
                expect = [int(partner[g, w]) for g in range(M) if f[g] and partner[g, w] >= 0]
                got = [row_base + s if s < n_local else senders[s - n_local] for s in src[r]]
                assert got == expect
            X = O.decen_round(X, partner, f, alpha)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchange_contract_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res[r] == "ok", res[r]
