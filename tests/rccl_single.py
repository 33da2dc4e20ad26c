"""One rank, real RCCL (torchrun --nproc-per-node 1, backend nccl): the library's own RCCL
communicator is created through RcclComm (unique id broadcast over torch.distributed), runs
mx_allreduce_mean, an exchange round with nothing to move, and a full VirtualWorkerGroup /
ChocoWorkerGroup round with the RCCL comm attached, then is destroyed.  This is the linkage check of
the N > 1 transport (the library binds to the RCCL torch already loaded); cross-GPU traffic itself
needs one GPU per rank."""
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
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
PKG = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    pkg = importlib.import_module(PKG)
    import oracle as O
    comm = pkg.engine.RcclComm()
    out = {"rank": comm.rank, "nranks": comm.nranks, "nonblocking": comm.nonblocking}
    # all-reduce mean over one rank: sum / 1 leaves every value as it was
    x = torch.from_numpy(O.synth(5, 1_000_003)).cuda()
    y = x.clone()
    pkg._lib.check(pkg.lib.mx_allreduce_mean(comm.handle, y.data_ptr(), y.numel(), 1, pkg._lib.stream_ptr()))
    torch.cuda.synchronize()
    out["allreduce_identity"] = bool(torch.equal(x, y))
    # gossip rounds with the RCCL communicator attached (one rank: no cross-GPU edge, so the
    # exchange posts nothing) -- bit-exact vs the oracle
    n, P = 8, 50_001
    np.random.seed(1234)
    GP = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, 6, True)
    grp = pkg.VirtualWorkerGroup(GP, numel=P, rank=0, nranks=1, comm=comm)
    X = np.stack([O.synth(1234 + i, P) for i in range(n)])
    grp.rows.copy_(torch.from_numpy(X))
    partner = np.asarray(GP.neighbors_info, np.int32)
    for it in range(6):
        nrem = grp.engine.exchange(it, grp._row_ptrs, None, grp.ld * 4, P * 4)
        assert nrem == 0
        grp.step(it)
        X = O.decen_round(X, partner, np.asarray(GP.active_flags[it], np.uint8), GP.neighbor_weight)
    torch.cuda.synchronize()
    out["decen_bit_exact"] = bool(np.array_equal(grp.rows.cpu().numpy().view(np.uint32), X.view(np.uint32)))
    # real ncclSend / ncclRecv through mx_exchange_post: a one-rank communicator sends to itself
    # (sends and receives to one peer pair up in posting order), so slab slot 2 gets row 0, slot 0
    # gets row 2 and slot 1 row 1 -- the slab addressing, counts and grouping of the N > 1 path
    import ctypes
    P2 = 300_007
    rows = torch.from_numpy(np.stack([O.synth(900 + i, P2) for i in range(3)])).cuda()
    ld = P2 + 57
    slab = torch.full((3, ld), -7.0, device="cuda")
    ops = np.array([[0, 0, 0, 0], [1, 0, 2, 0], [0, 0, 2, 2], [1, 0, 0, 2], [0, 0, 1, 1], [1, 0, 1, 1]],
                   np.int32)
    ptrs = (ctypes.c_void_p * 3)(*[rows[i].data_ptr() for i in range(3)])
    pkg._lib.check(pkg.lib.mx_exchange_post(comm.handle, ops.ctypes.data, len(ops), ptrs, 3, slab.data_ptr(),
                                            ld * 4, P2 * 4, pkg._lib.stream_ptr()))
    torch.cuda.synchronize()
    out["post_self_exchange"] = bool(torch.equal(slab[2, :P2], rows[0]) and torch.equal(slab[0, :P2], rows[2])
                                     and torch.equal(slab[1, :P2], rows[1])
                                     and bool((slab[:, P2:] == -7.0).all()))
    bad = ops.copy()
    bad[0, 2] = 5                                    # row index out of range: refused before posting
    rc = pkg.lib.mx_exchange_post(comm.handle, bad.ctypes.data, len(bad), ptrs, 3, slab.data_ptr(), ld * 4,
                                  P2 * 4, pkg._lib.stream_ptr())
    out["post_validates"] = rc != 0
    bad = ops.copy()
    bad[1, 1] = 1                                    # peer 1 of a one-rank communicator: refused
    rc = pkg.lib.mx_exchange_post(comm.handle, bad.ctypes.data, len(bad), ptrs, 3, slab.data_ptr(), ld * 4,
                                  P2 * 4, pkg._lib.stream_ptr())
    out["post_validates_peer"] = rc != 0
    # the reference-order all-reduce mean (all-gather + mx_mean_rows): one rank -> x / 1 = x
    z = x.clone()
    gather = torch.empty_like(z)
    pkg._lib.check(pkg.lib.mx_allreduce_mean_ordered(comm.handle, z.data_ptr(), z.numel(), gather.data_ptr(), 0,
                                                     pkg._lib.stream_ptr()))
    torch.cuda.synchronize()
    out["allreduce_ordered_identity"] = bool(torch.equal(x, z) and torch.equal(gather, x))
    out["count"] = comm.count()                     # ncclCommCount (the bench line's rccl_ranks)
    comm.wait()                                     # a drained stream: returns at once
    # the deadline-bounded stream wait: a kernel that outlives the deadline stands in
    # for an RCCL kernel whose peer died after the connections existed -- MXError after the
    # deadline (not a hang), the communicator aborted, the stream drained afterwards
    torch.cuda._sleep(int(1e9))
    t = time.time()
    try:
        comm.wait(timeout_s=0.1)
        out["wait_deadline"] = False
    except pkg.MXError as e:
        out["wait_deadline"] = "did not drain" in str(e) and comm.handle is None
    out["wait_deadline_s_ok"] = time.time() - t >= 0.1
    comm.close()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
