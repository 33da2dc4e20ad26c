"""The pull round's snapshot copy: mx_snapshot_publish_rows (per-row strided sweep, the row set
tested on the device) against mx_snapshot_publish_mask (tile sweep, the row set from the host) at
publish_wgpc workgroups per CU, for R published rows of P fp32 (R = 8 / 3 / 1: every local row at
N = 1-style 8-row blocks, the N = 2 rank-0 share of graph 0, the N = 8 share).  Per variant,
interleaved REPS times: one event pair around 40 launches.  Bits: the snapshot rows equal the
source rows, unpublished rows untouched.  One JSON line per R.

    WGPC=0,4,5,6 REPS=3 python tools/publish_ab.py [P]
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
E = pkg.engine
L = pkg.lib
chk = pkg._lib.check
P = int(float(sys.argv[1])) if len(sys.argv) > 1 else 25_600_000
reps = int(os.environ.get("REPS", "3"))
wgpc = [int(x) for x in os.environ.get("WGPC", "0,4,5,6").split(",")]
ld = (P + 63) // 64 * 64
cols = (P + 3) // 4 * 4
saved = E.mix_tuning()
for R, n_local in ((8, 8), (3, 4), (1, 1)):
    n_global = 2 * n_local
    src = torch.empty((n_local, ld), dtype=torch.float32, device="cuda")
    for r in range(n_local):
        chk(L.mx_synth_fill(src[r].data_ptr(), P, 77 + r, None))
    dst = torch.zeros_like(src)
    # matching 0 pairs local row i with remote worker n_local + i for i < R; the rest idle
    part = np.full(n_global, -1, np.int32)
    for i in range(R):
        part[i], part[n_local + i] = n_local + i, i
    partner = torch.from_numpy(part[None, :]).cuda()
    flags = torch.ones(1, dtype=torch.uint8, device="cuda")
    mask = (1 << R) - 1
    variants = [("rows", None)] + [(f"mask_wgpc{w}", w) for w in wgpc]

    def run(v):
        name, w = v
        if w is None:
            chk(L.mx_snapshot_publish_rows(src.data_ptr(), ld, dst.data_ptr(), ld, cols, n_local, flags.data_ptr(),
                                           1, partner.data_ptr(), n_global, 0, None))
        else:
            chk(L.mx_snapshot_publish_mask(src.data_ptr(), ld, dst.data_ptr(), ld, cols, n_local, mask, None))

    res, ok = {v[0]: [] for v in variants}, {}
    for rep in range(reps):
        for v in (variants if rep % 2 == 0 else variants[::-1]):
            if v[1] is not None:
                E.set_mix_tuning(publish_wgpc=v[1])
            dst.zero_()
            run(v)
            torch.cuda.synchronize()
            ok[v[0]] = bool(torch.equal(dst[:R, :P], src[:R, :P]) and not dst[R:].any())
            for _ in range(5):
                run(v)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(40):
                run(v)
            b.record()
            torch.cuda.synchronize()
            res[v[0]].append(a.elapsed_time(b) / 40)
    byts = 2 * R * cols * 4
    out = {"P": P, "published_rows": R, "n_local": n_local, "bytes_per_launch": byts}
    for name, _ in variants:
        ms = min(res[name])
        out[name] = {"ms_min": round(ms, 4), "ms_all": [round(x, 4) for x in res[name]],
                     "frac_8TBps": round(byts / (ms * 1e-3) / 8e12, 4), "same_bits": ok[name]}
    print(json.dumps(out), flush=True)
    del src, dst
    torch.cuda.empty_cache()
E.set_mix_tuning(**saved)
