"""The pull round's snapshot publish, whole block vs only the rows a peer reads.

For every rank of the 2 / 4 / 8-GPU layouts of graph 0 (8 workers, placement "auto" as bench.py)
at the headline row size (P = 25.6M fp32), the per-launch time of
  all   -- mx_snapshot_publish of the rank's n_local rows (the round-5 round: every row, every round)
  rows  -- mx_snapshot_publish_rows driven by the round's flags (rows with an active partner on
           another GPU only)
over three kinds of round: every matching active ("full"), a MATCHA C_b = 0.5 schedule ("matcha":
its first 40 non-empty rounds) and each single matching alone ("single").  One process, one GPU:
publish is a per-rank kernel, so each rank's block is run in turn on the same GPU.  HIP events per
launch, median of the reps.  One JSON line.

    python tools/publish_rows.py [P]
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"


def main():
    pkg = importlib.import_module(PKG)
    L, chk = pkg.lib, pkg._lib.check
    P = int(float(sys.argv[1])) if len(sys.argv) > 1 else 25_600_000
    ld = (P + 63) // 64 * 64
    cols = (P + 3) // 4 * 4
    n = 8
    np.random.seed(1234)
    gpm = pkg.MatchaProcessor(pkg.select_graph(0), 0.5, 0, n, 400, True)
    fl = np.asarray(gpm.active_flags, np.uint8)
    matcha_rows = [f for f in fl if f.any()][:40]
    M = fl.shape[1]
    kinds = {"full": [np.ones(M, np.uint8)], "matcha": matcha_rows,
             "single": [np.eye(M, dtype=np.uint8)[g] for g in range(M)]}
    src = torch.empty((4, ld), dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)
    src.uniform_()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def launch_ms(fn, reps=5):
        out = []
        for _ in range(reps):
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            out.append(ev[0].elapsed_time(ev[1]))
        return float(np.median(out))

    res = {"P": P, "layouts": {}}
    for world in (2, 4, 8):
        topo, perm = pkg.placement.place(gpm, world, "auto")
        partner = np.ascontiguousarray(np.asarray(topo.neighbors_info, np.int32).reshape(-1, n)[:M])
        part_dev = torch.from_numpy(partner).cuda()
        ranks = []
        for rank, (rb, nl) in enumerate(pkg.partition(n, world)):
            all_ms = launch_ms(lambda: chk(L.mx_snapshot_publish(src.data_ptr(), dst.data_ptr(), nl * ld, None)))
            row = {"rank": rank, "rows": nl, "all_ms": all_ms}
            for kind, rows in kinds.items():
                ms, nrow = [], []
                for f in rows:
                    fd = torch.from_numpy(f).cuda()
                    ms.append(launch_ms(lambda: chk(L.mx_snapshot_publish_rows(
                        src.data_ptr(), ld, dst.data_ptr(), ld, cols, nl, fd.data_ptr(), M, part_dev.data_ptr(), n, rb,
                        None))))
                    nrow.append(sum(1 for r in range(rb, rb + nl)
                                    if any(f[g] and partner[g, r] >= 0 and not (rb <= partner[g, r] < rb + nl)
                                           for g in range(M))))
                row[kind] = {"rows_ms_mean": float(np.mean(ms)), "rows_published_mean": float(np.mean(nrow)),
                             "vs_all": float(np.mean(ms)) / all_ms}
            ranks.append(row)
        res["layouts"][world] = {"placement": [int(x) for x in perm] if perm is not None else "identity", "ranks": ranks}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
