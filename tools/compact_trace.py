"""Where the one-row Choco compaction's time goes (lever 2): ramp or tail?

One row of the VGG-16 share (P = 14,774,436, top-1 %: k = 147,744), x_hat = x minus a small drift so
the floor and candidate count are the Choco round's.  With mx_topk_set("compact_trace", 1) every
compaction workgroup stamps the 100 MHz constant clock at its start, once its floor is resolved and
at its end (mx_topk_trace).  Over REPS calls: the launch span (first start -> last end), the spread
of the starts (dispatch ramp), the per-block prologue (start -> floor), the spread of the ends (tail)
and the median block's span; plus the HIP-event time of the whole call and of a compaction-only
share estimate.  Prints one JSON line."""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
L = pkg.lib
P = int(os.environ.get("TRACE_P", 14_774_436))
ratio = float(os.environ.get("TRACE_RATIO", 0.99))
reps = int(os.environ.get("REPS", 20))
k = max(1, int(P * (1 - ratio)))
x = torch.empty(P, dtype=torch.float32, device="cuda")
xh = torch.empty(P, dtype=torch.float32, device="cuda")
pkg._lib.check(L.mx_synth_fill(x.data_ptr(), P, 1234, None))
pkg._lib.check(L.mx_synth_fill(xh.data_ptr(), P, 99, None))
xh.mul_(0.01).add_(x)                         # x_hat close to x: |x - x_hat| ~ 0.01 uniform
vals = torch.empty(k, dtype=torch.float32, device="cuda")
idx = torch.empty(k, dtype=torch.int64, device="cuda")
work = torch.zeros(int(L.mx_topk_work_bytes(P)), dtype=torch.uint8, device="cuda")
for kv in filter(None, os.environ.get("TOPK_SET", "").split(":")):     # e.g. TOPK_SET=compact_dyn=1
    k_, v_ = kv.split("=")
    pkg._lib.check(L.mx_topk_set(k_.encode(), int(v_)))
call = lambda: pkg._lib.check(L.mx_topk_abs_diff(x.data_ptr(), xh.data_ptr(), P, k, vals.data_ptr(), idx.data_ptr(),
                                                 work.data_ptr(), None))
nc = (P + 4095) // 4096
q = max(1, (nc + 360) // 720)
nb = (nc + q - 1) // q                         # the one-row auto grid (choco.hip)
for _ in range(5):
    call()
torch.cuda.synchronize()
ev_ms = []
for _ in range(reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    call()
    b.record()
    torch.cuda.synchronize()
    ev_ms.append(a.elapsed_time(b))
pkg._lib.check(L.mx_topk_set(b"compact_trace", 1))
stats = []
buf = np.zeros(3 * nb, np.uint64)
for _ in range(reps):
    call()
    pkg._lib.check(L.mx_topk_trace(buf.ctypes.data, nb))
    t = buf.reshape(nb, 3).astype(np.int64)
    t0 = t[:, 0].min()
    st, fl, en = (t[:, 0] - t0) * 10e-3, (t[:, 1] - t0) * 10e-3, (t[:, 2] - t0) * 10e-3   # us
    stats.append({"span": en.max(), "start_p50": np.median(st), "start_max": st.max(),
                  "prologue_p50": np.median(fl - st), "prologue_max": (fl - st).max(),
                  "block_p50": np.median(en - st), "block_max": (en - st).max(),
                  "end_min": en.min(), "end_p50": np.median(en), "end_p90": np.percentile(en, 90),
                  "last_start_block_end": en[np.argmax(st)]})
pkg._lib.check(L.mx_topk_set(b"compact_trace", 0))
med = {key: round(float(np.median([s[key] for s in stats])), 2) for key in stats[0]}
chunks = nc
print(json.dumps({"lib": os.environ.get("MX_GOSSIP_LIB") or "tree", "topk_set": os.environ.get("TOPK_SET", ""), "P": P, "k": k, "chunks": chunks, "blocks": nb, "chunks_per_block": q,
                  "call_us_median_events": round(1e3 * float(np.median(ev_ms)), 2),
                  "compaction_trace_us_median": med,
                  "bytes": 8 * P, "TBps_over_span": round(8 * P / (med["span"] * 1e-6) / 1e12, 3),
                  "TBps_over_block_p50": round(8 * P / (med["block_p50"] * 1e-6) / 1e12, 3),
                  "note": "times in us from the first block's start; stamps of the 100 MHz constant clock"}))
