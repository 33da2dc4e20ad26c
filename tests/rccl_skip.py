"""Two ranks, one GPU each, real RCCL (torchrun --nproc-per-node 2): both run one all-gather (the
connections now exist), then rank 1 skips the second one and idles.  Rank 0's RcclComm.wait()
(mx_rccl_wait: the stream polled against a deadline) must raise MXError "did not drain" after
its 3 s deadline -- the communicator aborted -- instead of hanging in a stream synchronisation
(a peer that dies or skips an exchange after the connections exist).  Rank 0
prints one JSON line."""
import importlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
PKG = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = importlib.import_module(PKG)
    comm = pkg.engine.RcclComm(timeout_s=30)
    n = 1 << 20
    send = torch.full((n,), float(rank + 1), device="cuda")
    gather = torch.empty(world * n, device="cuda")
    pkg._lib.check(pkg.lib.mx_allgather(comm.handle, send.data_ptr(), n, gather.data_ptr(), pkg._lib.stream_ptr()))
    comm.wait(timeout_s=30)
    first_ok = bool((gather.view(world, n)[:, 0].cpu() == torch.arange(1, world + 1, dtype=torch.float32)).all())
    dist.barrier()
    if rank == 1:
        time.sleep(12)                               # skips the second all-gather, then leaves
        return
    pkg._lib.check(pkg.lib.mx_allgather(comm.handle, send.data_ptr(), n, gather.data_ptr(), pkg._lib.stream_ptr()))
    t = time.time()
    err = None
    try:
        comm.wait(timeout_s=3)
    except pkg.MXError as e:
        err = str(e)
    print(json.dumps({"first_ok": first_ok, "error": err, "seconds": time.time() - t,
                      "aborted": comm.handle is None}), flush=True)
    os._exit(0)                                      # the aborted communicator is not finalised


if __name__ == "__main__":
    main()
