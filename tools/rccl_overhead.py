"""RCCL's per-round fixed cost as far as one GPU can show it (the `predicted` object's RCCL term,
DESIGN.md §6): one rank (torchrun --nproc-per-node 1, backend nccl), the library's own RCCL
communicator, mx_exchange_post of a send + receive to ITSELF inside one group (RCCL's self
transport: a copy on this GPU, no xGMI), K rounds back to back, for message sizes from 4 KB to a
headline row.  The small-message round time is RCCL's group launch + protocol cost -- a lower bound
of what a two-GPU exchange pays before its bytes move.  Prints one JSON line."""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    pkg = importlib.import_module(PKG)
    comm = pkg.engine.RcclComm()
    K = int(os.environ.get("K", 100))
    res = {"K": K, "rounds": []}
    for nbytes in (4096, 1 << 20, 1_772_944, 16 << 20, 102_400_000):
        n = nbytes // 4
        row = torch.zeros(n, dtype=torch.float32, device="cuda")
        slab = torch.empty(n, dtype=torch.float32, device="cuda")
        ops = np.array([[0, 0, 0, 0], [1, 0, 0, 0]], np.int32)
        ptrs = (ctypes.c_void_p * 1)(row.data_ptr())
        post = lambda: pkg._lib.check(pkg.lib.mx_exchange_post(comm.handle, ops.ctypes.data, 2, ptrs, 1, slab.data_ptr(),
                                                               n * 4, n * 4, pkg._lib.stream_ptr()))
        for _ in range(10):
            post()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        a.record()
        for _ in range(K):
            post()
        b.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / K
        # one round at a time (host waits each round): launch latency included
        t = time.perf_counter()
        for _ in range(20):
            post()
            torch.cuda.synchronize()
        single = (time.perf_counter() - t) / 20
        res["rounds"].append({"bytes": nbytes, "us_per_round_back_to_back_events": round(1e3 * a.elapsed_time(b) / K, 2),
                              "us_per_round_back_to_back_wall": round(1e6 * wall, 2),
                              "us_per_round_synchronized": round(1e6 * single, 2)})
        del row, slab
    comm.close()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
