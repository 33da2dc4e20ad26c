"""Does mx_ipc_alloc (hipMalloc + hipIpcGetMemHandle) fail for some small sizes once the process has
made other allocations?  Interleaves torch allocations of assorted sizes with IPC allocations of
assorted sizes, unrounded vs rounded up to 2 MiB, and counts hipIpcGetMemHandle failures.  One JSON
line."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
L = pkg.lib
hb = int(L.mx_ipc_handle_bytes())
rng = np.random.RandomState(0)
res = {}
for mode in ("exact", "round2m"):
    fails, total, msgs = 0, 0, set()
    keep, held = [], []
    for i in range(400):
        keep.append(torch.empty(int(rng.randint(1, 4 << 20)), dtype=torch.uint8, device="cuda"))
        if len(keep) > 50:
            keep.pop(rng.randint(len(keep)))
        nbytes = int(rng.choice([600_000, 1_600_000, 3_200_000, 256 + 2 * 4 * 20032 * 4, 256 + 2 * 4 * 50048 * 4,
                                 17_000, 1 << 20]))
        if mode == "round2m":
            nbytes = (nbytes + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        p, h = ctypes.c_void_p(), (ctypes.c_char * hb)()
        rc = L.mx_ipc_alloc(nbytes, ctypes.byref(p), ctypes.cast(h, ctypes.c_void_p))
        total += 1
        if rc:
            fails += 1
            msgs.add(L.mx_last_error().decode()[:120])
        else:
            held.append(p.value)
            if len(held) > 8:
                L.mx_ipc_free(held.pop(0))
    for q in held:
        L.mx_ipc_free(q)
    res[mode] = {"allocs": total, "fails": fails, "errors": sorted(msgs)}
print(json.dumps(res), flush=True)
