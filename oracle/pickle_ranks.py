"""CPU baseline: the reference's per-rank gossip sequence with a PICKLED transport, one process
per worker, each pinned to its own host core -- what `mpirun -np 8 python train_mpi.py` spends
per decenCommunicator round (communicator.py:87-131), restated in torch + multiprocessing.

TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg runs it; the product package
never imports it.  The reference itself cannot run here (no MPI runtime, no mpi4py) and never
travels to the GPU box, so this is a restatement (kind "port"), faithful in the parts that cost:

  flatten_tensors: torch.cat of the model's tensors           comm_helpers.py:27-30
  recv_buffer = zeros_like                                      communicator.py:90
  comm.barrier() before averaging                               communicator.py:94
  per active matching, partner j: comm.sendrecv(send_buffer)    communicator.py:110
      = pickle.dumps(tensor) -> OS pipe -> pickle.loads on the partner (mpi4py's lowercase API
        pickles the object; its shared-memory transport is a byte copy like the pipe)
      recv_buffer.add_(recv_tmp, alpha=alpha)                   communicator.py:112
  recv_buffer.add_(send_buffer, alpha=1 - degree * alpha)       communicator.py:117
  comm.barrier()                                                communicator.py:119
  reset_model: unflatten views, t.copy_(f)                      communicator.py:124-131

Blocking pairwise exchange without deadlock: both partners walk matchings in the same order
(like the reference), the lower rank sends first and the higher receives first.
"""
import multiprocessing as mp
import os
import pickle
import time

import numpy as np

TENSOR_SPLIT = 54       # the model's parameter count is split into this many tensors (VGG-16 has 54)


def _segments(P, nseg):
    cuts = np.linspace(0, P, nseg + 1).astype(np.int64)
    return [(int(a), int(b)) for a, b in zip(cuts[:-1], cuts[1:])]


def _rank_main(rank, n, P, partner, flags, alpha, conns, core, barrier, out_q, nseg=TENSOR_SPLIT):
    import torch
    try:
        os.sched_setaffinity(0, {core})
    except (AttributeError, OSError):
        pass
    torch.set_num_threads(1)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle as O
    row = O.synth(1234 + rank, P)
    tensors = [torch.from_numpy(row[a:b].copy()) for a, b in _segments(P, nseg)]
    del row
    M = partner.shape[0]
    barrier.wait()
    t0 = time.perf_counter()
    for f in flags:
        if not f.any():                                   # communicator.py:140-141
            continue
        send = torch.cat([t.reshape(-1) for t in tensors])
        recv = torch.zeros_like(send)
        barrier.wait()
        degree = 0
        for g in range(M):
            if not f[g]:
                continue
            j = int(partner[g, rank])
            if j == -1:
                continue
            degree += 1
            c = conns[j]
            if rank < j:
                c.send_bytes(pickle.dumps(send, protocol=pickle.HIGHEST_PROTOCOL))
                tmp = pickle.loads(c.recv_bytes())
            else:
                tmp = pickle.loads(c.recv_bytes())
                c.send_bytes(pickle.dumps(send, protocol=pickle.HIGHEST_PROTOCOL))
            recv.add_(tmp, alpha=alpha)
            del tmp
        recv.add_(send, alpha=1 - degree * alpha)
        barrier.wait()
        off = 0
        with torch.no_grad():
            for t in tensors:
                t.copy_(recv[off:off + t.numel()].view_as(t))
                off += t.numel()
    barrier.wait()
    el = time.perf_counter() - t0
    out_q.put((rank, el, float(tensors[0][0]), float(tensors[-1][-1])))


def run(partner, flags, alpha, P, cores=None, nseg=TENSOR_SPLIT):
    """Rounds given by `flags` ([rounds][M] uint8) over n = partner.shape[1] worker processes, each
    model's P parameters in `nseg` tensors.  Returns (seconds for all rounds, max over ranks; cores
    used; first/last element per rank)."""
    partner = np.ascontiguousarray(partner, np.int32)
    flags = np.ascontiguousarray(flags, np.uint8)
    n = partner.shape[1]
    avail = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    cores = list(cores) if cores is not None else [avail[i % len(avail)] for i in range(n)]
    ctx = mp.get_context("spawn")
    ends = {i: {} for i in range(n)}
    for g in range(partner.shape[0]):
        for i in range(n):
            j = int(partner[g, i])
            if j > i and j not in ends[i]:
                a, b = ctx.Pipe(duplex=True)
                ends[i][j], ends[j][i] = a, b
    barrier = ctx.Barrier(n)
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, n, P, partner, flags, float(alpha), ends[r], cores[r],
                                                  barrier, q, int(nseg)), daemon=True) for r in range(n)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=900) for _ in range(n)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    res.sort()
    return max(r[1] for r in res), len(set(cores)), [(r[2], r[3]) for r in res]
