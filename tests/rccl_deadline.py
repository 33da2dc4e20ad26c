"""One process, real RCCL: a communicator of 2 ranks whose second rank never joins.

mx_rccl_init_timeout creates the communicator non-blocking and polls it against a deadline, so
the missing peer (a dead rank, or one that skipped the call) turns into MX_ERR_RCCL "timed out"
after the deadline instead of a hang (VERDICT r02 "hang-proof the N > 1 path").  Prints one JSON
line: the status, the message and the seconds the call took."""
import ctypes
import importlib
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
PKG = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"


def main():
    torch.cuda.set_device(0)
    pkg = importlib.import_module(PKG)
    uid = (ctypes.c_char * 128)()
    pkg._lib.check(pkg.lib.mx_rccl_unique_id(ctypes.cast(uid, ctypes.c_void_p)))
    h, nb = ctypes.c_void_p(), ctypes.c_int(0)
    t = time.time()
    rc = pkg.lib.mx_rccl_init_timeout(ctypes.cast(uid, ctypes.c_void_p), 2, 0, 4000, ctypes.byref(h),
                                      ctypes.byref(nb))
    el = time.time() - t
    print(json.dumps({"rc": int(rc), "seconds": el, "handle_null": h.value is None,
                      "message": pkg.lib.mx_last_error().decode()}), flush=True)


if __name__ == "__main__":
    main()
