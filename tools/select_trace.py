"""Stage clocks of select_kernel (mx_topk_set "select_trace"): one row of P (default the VGG-16
share, 14,774,436) with x - x_hat from two synthetic rows, a few warm calls, then per stage the
min / median / max over the row's blocks of the constant-clock stamp (us after the earliest block
start).  Stages: 0 start, 1 12-bit resolved (cache loaded), 2 pass 1 done, 3 barrier 1 passed,
4 10-bit resolved, 5 pass 2 done, 6 barrier 2 passed, 7 threshold + bases resolved, 8 written."""
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

P = int(os.environ.get("CHOCO_P", 14_774_436))
B = int(os.environ.get("SEL_B", 32))
k = max(1, int(P * 0.01))
nc = (P + 4095) // 4096
a256 = lambda v: (v + 255) // 256 * 256
hist_words = 3 * 4096 + 1024 + 512
cnt = 4 * hist_words + 64
cval = a256(cnt + 2 * 64 * nc)
cloc = cval + 4 * nc * (4096 + 64)
pub = a256(cloc + 2 * nc * (4096 + 128))
pub9 = pub + 4 * 32 * 1024
wb = int(L.mx_topk_work_bytes(P))
assert wb == pub + 4 * 32 * (1024 + 528), (wb, pub)

x = torch.empty(P, dtype=torch.float32, device="cuda")
xh = torch.empty(P, dtype=torch.float32, device="cuda")
pkg._lib.check(L.mx_synth_fill(x.data_ptr(), P, 1234, None))
pkg._lib.check(L.mx_synth_fill(xh.data_ptr(), P, 99, None))
xh.mul_(0.999)
kpad = (k + 1) // 2 * 2
nb = int(L.mx_choco_msg_bytes(P, k))
out = torch.zeros(nb, dtype=torch.uint8, device="cuda")
work = torch.zeros(wb, dtype=torch.uint8, device="cuda")
pkg._lib.check(L.mx_topk_set(b"select", 1))
pkg._lib.check(L.mx_topk_set(b"select_blocks", B))


def call():
    pkg._lib.check(L.mx_topk_abs_diff_rows(x.data_ptr(), xh.data_ptr(), P, 1, P, k, out.data_ptr(), 0, 4 * kpad,
                                           4 * kpad + 8 * k, work.data_ptr(), 0, None), "topk")


for _ in range(10):
    call()
pkg._lib.check(L.mx_topk_set(b"select_trace", 1))
stamps = []
for rep in range(int(os.environ.get("REPS", 5))):
    call()
    torch.cuda.synchronize()
    w = work.cpu().numpy()
    st = np.stack([w[pub9 + 4 * (b * 528 + 513):pub9 + 4 * (b * 528 + 522)].view(np.uint32) for b in range(B)])
    st = (st.astype(np.int64) - int(st[:, 0].min())) * 0.01     # 100 MHz ticks -> us
    stamps.append(st)
    for _ in range(3):
        call()
pkg._lib.check(L.mx_topk_set(b"select_trace", 0))
s = np.median(np.stack(stamps), axis=0)                      # [B][9], median over reps
names = ["start", "resolved12", "pass1", "barrier1", "resolved10", "pass2", "barrier2", "bases", "written"]
for i, n in enumerate(names):
    print(json.dumps({"stage": i, "name": n, "min_us": round(float(s[:, i].min()), 2),
                      "median_us": round(float(np.median(s[:, i])), 2), "max_us": round(float(s[:, i].max()), 2)}))
