"""Where the headline round's time goes between launches (VERDICT r01 "kernel vs driver clock").

Headline shape (graph 0, 8 workers x 25.6M fp32, every matching active).  For each mixing-kernel
variant it times, on one stream:
  * per-launch HIP events (the kernel's own duration),
  * K launches back to back bracketed by ONE event pair (kernel + inter-launch gap),
  * the same K launches on the host clock with synchronize on both sides (the bench's clock).
Run it under `rocprofv3 --kernel-trace` and pass the kernel_trace.csv to `--trace` afterwards to
get start[i+1] - end[i] for consecutive mixing launches.

    python tools/gaps.py [K] [grid=...] ...
    python tools/gaps.py --trace path/kernel_trace.csv
"""
import csv
import importlib
import json
import os
import sys
import time

import numpy as np


def trace_gaps(path, K=20):
    """All mixing launches of a kernel trace, and bench.py's timed region: the first run of >= K
    launches of the headline kernel with no event between them (gaps < 3 us) -- the warmup is
    shorter than K and the settling blocks put an event pair around every launch, so the first
    such run is the K timed rounds (the MATCHA figure's back-to-back rounds come later)."""
    allrows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    mixrows = [r for r in allrows if "mix_kernel" in r["Kernel_Name"]]
    timed = None
    if mixrows:
        hk = max({r["Kernel_Name"] for r in mixrows}, key=lambda nm: sum(r["Kernel_Name"] == nm for r in mixrows))
        head = [r for r in mixrows if r["Kernel_Name"] == hk]
        run = [head[0]]
        for a, b in zip(head, head[1:]):
            if (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 < 3.0:
                run.append(b)
                continue
            if len(run) >= K:
                break
            run = [b]
        if len(run) >= K:
            run = run[:K]
            st = np.array([int(r["Start_Timestamp"]) for r in run], np.int64)
            en = np.array([int(r["End_Timestamp"]) for r in run], np.int64)
            timed = {"launches": K, "kernel": hk[:80], "kernel_us_mean": float(((en - st) / 1e3).mean()),
                     "gaps_us": [round(float(g), 3) for g in (st[1:] - en[:-1]) / 1e3],
                     "span_us_per_round": float((en[-1] - st[0]) / 1e3 / K)}
    rows = [r for r in allrows if "mix_kernel" in r["Kernel_Name"]]
    st = np.array([int(r["Start_Timestamp"]) for r in rows], np.int64)
    en = np.array([int(r["End_Timestamp"]) for r in rows], np.int64)
    dur = (en - st) / 1e3
    gap = (st[1:] - en[:-1]) / 1e3
    gap = gap[gap < 50]            # consecutive launches of one back-to-back run only
    print(json.dumps({"launches": len(rows), "dur_us_median": float(np.median(dur)), "dur_us_min": float(dur.min()),
                      "gap_us_median": float(np.median(gap)) if len(gap) else None,
                      "gap_us_p10_p90": [float(np.percentile(gap, 10)), float(np.percentile(gap, 90))] if len(gap) else None,
                      "gaps_counted": int(len(gap)), "timed_region": timed,
                      "note": "all mixing launches incl. per-round-event diagnostic blocks (events between "
                              "launches) and the mixing-alone event timing; timed_region = bench.py's K "
                              "back-to-back rounds"}))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--trace":
        return trace_gaps(sys.argv[2])
    import torch
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    pkg = importlib.import_module("270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd")
    from conftest import Topo

    K = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 50
    variants = [a for a in sys.argv[1:] if "=" in a] or ["default"]
    n, P = 8, 25_600_000
    gp = pkg.GraphProcessor(pkg.select_graph(0), 1.0, 0, n, 4, True)
    topo = Topo(gp.neighbors_info, 2 / 7, np.ones((4 * K + 64, 5), np.uint8))
    grp = pkg.VirtualWorkerGroup(topo, numel=P)
    for i in range(n):
        pkg.lib.mx_synth_fill(grp.rows[i].data_ptr(), P, 1234 + i, None)
    nbytes = 2 * n * P * 4
    base = pkg.engine.mix_tuning()
    for v in variants:
        knobs = dict(base)
        if v != "default":
            for kv in v.split(","):
                k, x = kv.split("=")
                knobs[k] = int(x)
        pkg.engine.set_mix_tuning(**knobs)
        lay = pkg.Layout([P], [[grp.arena[r].data_ptr()] for r in range(n)], grp.engine.n_slots)
        mix = lambda j: grp.engine.mix(j, lay)
        for j in range(20):                       # warm the clocks
            mix(j)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for j, (a, b) in enumerate(ev):
            a.record()
            mix(j)
            b.record()
        torch.cuda.synchronize()
        per = np.array([a.elapsed_time(b) for a, b in ev]) * 1e3
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for j in range(K):
            mix(j)
        b.record()
        torch.cuda.synchronize()
        b2b = a.elapsed_time(b) * 1e3 / K
        torch.cuda.synchronize()
        t = time.perf_counter()
        for j in range(K):
            mix(j)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e6 / K
        print(json.dumps({"variant": v, "K": K, "kernel_us_median": float(np.median(per)), "kernel_us_min": float(per.min()),
                          "kernel_us_mean": float(per.mean()), "b2b_events_us": b2b, "b2b_wall_us": wall,
                          "gap_us": b2b - float(per.mean()), "frac_wall": nbytes / (wall * 1e-6) / 8e12}), flush=True)
    pkg.engine.set_mix_tuning(**base)


if __name__ == "__main__":
    main()
