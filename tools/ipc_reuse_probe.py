"""Pins the cause of the recorded hipIpcGetMemHandle refusals ("invalid argument" on a fresh
mx_ipc_alloc block in a long multi-process run; rounds 5 and 6).  First hypothesis: the exporter
freed its previous buffer while a peer still held the import.  Result
(profiles/r06t_ipc_reuse_probe.json): no -- the refusals follow this process CLOSING a peer's import
(hipIpcCloseMemHandle) before it allocates: the new block lands on the released address range.

Two ranks (torchrun, both on GPU 0), ITERS rounds per mode and size; every round each rank allocates
and exports a block, imports the peer's, then:
  unsafe     -- rank 0 frees its block and allocates + exports the same size again while its import
                of the peer's block is still open (the peer waits HOLD_S before closing);
  safe       -- every rank closes its imports, a barrier, every rank frees its block, then rank 0
                allocates + exports again (the close() -> next bind() sequence);
  safe_sync  -- the same with a device synchronize after the closes;
  safe_sleep -- the same with a 50 ms sleep after the closes;
  safe_hold  -- "safe" with mx_ipc_alloc's hold-and-reallocate on (a refused block is kept while a
                second one is allocated and exported); the other modes run with it off.
Rank 0 prints one JSON line: final refusals per mode and size, and the recovered count.

    MODES=unsafe,safe,safe_hold python -m torch.distributed.run --nproc-per-node 2 \
        --master-addr 127.0.0.1 tools/ipc_reuse_probe.py
"""
import ctypes
import importlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
L = pkg.lib


def alloc(n):
    hb = int(L.mx_ipc_handle_bytes())
    own, h = ctypes.c_void_p(), (ctypes.c_char * hb)()
    rc = L.mx_ipc_alloc(n, ctypes.byref(own), ctypes.cast(h, ctypes.c_void_p))
    return rc, own.value, bytes(h)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    iters = int(os.environ.get("ITERS", "20"))
    hold = float(os.environ.get("HOLD_S", "0.2"))
    sizes = [int(x) for x in os.environ.get("SIZES", "1000,2097152,4194304").split(",")]
    out = {"iters": iters, "hold_s": hold}
    modes = os.environ.get("MODES", "unsafe,safe,safe_sync,safe_sleep,safe_hold").split(",")
    for m in modes:
        out[m] = {}
    for mode in modes + modes:
        L.mx_ipc_set(b"hold", 1 if mode == "safe_hold" else 0)
        for n in sizes:
            refused = 0
            for _ in range(iters):
                rc, own, h = alloc(n)
                hs = [None] * world
                dist.all_gather_object(hs, (rc, h))
                imports = []
                if all(r == 0 for r, _ in hs):
                    for r, (_, hh) in enumerate(hs):
                        if r == rank:
                            continue
                        buf = (ctypes.c_char * len(hh)).from_buffer_copy(hh)
                        p = ctypes.c_void_p()
                        pkg._lib.check(L.mx_ipc_open(ctypes.cast(buf, ctypes.c_void_p), ctypes.byref(p)), "mx_ipc_open")
                        imports.append(p.value)
                dist.barrier()
                if mode == "unsafe":
                    if rank == 0:
                        if own:
                            L.mx_ipc_free(own)
                        rc2, own2, _ = alloc(n)              # the same size again, peer's import still open
                        refused += rc2 != 0
                        if own2:
                            L.mx_ipc_free(own2)
                    else:
                        time.sleep(hold)
                    for p in imports:
                        L.mx_ipc_close(p)
                    if rank != 0 and own:
                        L.mx_ipc_free(own)
                else:
                    for p in imports:
                        L.mx_ipc_close(p)
                    if mode == "safe_sync":
                        torch.cuda.synchronize()
                    elif mode == "safe_sleep":
                        time.sleep(0.05)
                    dist.barrier()                           # every import closed before any free
                    if own:
                        L.mx_ipc_free(own)
                    if rank == 0:
                        rc2, own2, _ = alloc(n)
                        refused += rc2 != 0
                        if own2:
                            L.mx_ipc_free(own2)
                dist.barrier()
            tot = [None] * world
            dist.all_gather_object(tot, refused)
            out[mode][str(n)] = out[mode].get(str(n), 0) + sum(tot)
    ex, ref = pkg.engine.ipc_stats()
    out["exports"], out["refused_total"], out["recovered"] = ex, ref, int(L.mx_ipc_get(b"recovered"))
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
