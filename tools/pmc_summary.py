"""Summarise rocprofv3 CSV output (kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes) into one
JSON file under profiles/.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE
reports exactly half of the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def pick(d, *names):
    for n in names:
        if n in d and d[n] != "":
            return d[n]
    raise KeyError(names)


def counter_per_kernel(path, counter):
    acc = {}
    for r in rows(os.path.join(path, "**", "*counter_collection.csv")):
        if pick(r, "Counter_Name", "Counter-Name") != counter:
            continue
        name = pick(r, "Kernel_Name", "Kernel-Name")
        acc.setdefault(name, []).append(float(pick(r, "Counter_Value", "Counter-Value")))
    return acc


def summarize(src, trace="trace", fetch_dir="fetch", write_dir="write"):
    """kernel stats + per-launch HBM bytes of one profiled process tree under `src`"""
    stats = rows(os.path.join(src, trace, "**", "*kernel_stats.csv"))
    kernels = {}
    for r in stats:
        name = pick(r, "Name", "KernelName")
        kernels[name] = {"calls": int(pick(r, "Calls")), "avg_us": float(pick(r, "AverageNs")) / 1e3,
                         "min_us": float(pick(r, "MinNs")) / 1e3, "max_us": float(pick(r, "MaxNs")) / 1e3,
                         "pct": float(pick(r, "Percentage"))}
    fetch = counter_per_kernel(os.path.join(src, fetch_dir), "FETCH_SIZE")
    write = counter_per_kernel(os.path.join(src, write_dir), "WRITE_SIZE")
    mix = {}
    for name in set(fetch) | set(write):
        if "mix_kernel" not in name:
            continue
        f = fetch.get(name, [])
        w = write.get(name, [])
        f_kib = sum(f) / len(f) if f else None
        w_kib = sum(w) / len(w) if w else None
        mix[name] = {
            "launches_fetch": len(f), "launches_write": len(w),
            "FETCH_SIZE_KiB_avg": f_kib, "WRITE_SIZE_KiB_avg": w_kib,
            "hbm_read_bytes_corrected": 2 * 1024 * f_kib if f_kib is not None else None,
            "hbm_write_bytes": 1024 * w_kib if w_kib is not None else None,
        }
        if f_kib is not None and w_kib is not None:
            mix[name]["hbm_bytes_per_launch"] = 2 * 1024 * f_kib + 1024 * w_kib
    allk = {}
    for name in set(fetch) | set(write):
        f = fetch.get(name, [])
        w = write.get(name, [])
        if not f or not w:
            continue
        allk[name] = {"launches": min(len(f), len(w)),
                      "hbm_read_bytes_corrected": 2 * 1024 * sum(f) / len(f),
                      "hbm_write_bytes": 1024 * sum(w) / len(w),
                      "hbm_bytes_per_launch": 2 * 1024 * sum(f) / len(f) + 1024 * sum(w) / len(w)}
    return {"kernels": kernels, "mix_pmc": mix, "pmc_all": allk}


def summarize_ranks(src):
    """tools/profile_multi.sh layout: <pass>/rank<R>/... per rank (or, where this rocprofv3 did not
    expand %env{RANK}%, one directory per process id).  Per rank: the summary above, the RCCL kernels'
    share of the trace, and the xGMI bytes per launch of every kernel (fabric_gmi/ pass)."""
    out = {}
    ranks = sorted({d.split("rank", 1)[1] for d in os.listdir(os.path.join(src, "trace")) if d.startswith("rank")})
    for r in ranks:
        rs = summarize(src, os.path.join("trace", "rank" + r), os.path.join("fetch_size", "rank" + r),
                       os.path.join("write_size", "rank" + r))
        rs["rccl_kernels"] = {k: v for k, v in rs["kernels"].items() if "nccl" in k.lower() or "rccl" in k.lower()}
        # xGMI: 32-byte fabric requests to another GPU's memory, per launch of every kernel
        fab = {}
        for c, what in (("TCC_EA0_RDREQ_GMI_32B_sum", "read"), ("TCC_EA0_WRREQ_WRITE_GMI_32B_sum", "write")):
            per = counter_per_kernel(os.path.join(src, "fabric_gmi", "rank" + r), c)
            for k, v in per.items():
                if v:
                    fab.setdefault(k, {"launches": len(v)})[f"xgmi_{what}_bytes_per_launch"] = 32 * sum(v) / len(v)
        rs["xgmi_per_kernel"] = fab
        out["rank" + r] = rs
    return out


def main(src, dst, ranks=False):
    out = {"source": src}
    if ranks:
        out["ranks"] = summarize_ranks(src)
    else:
        out.update(summarize(src))
    out["note"] = "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes x1024"
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    for tag, rs in (out["ranks"].items() if ranks else [("", out)]):
        top = sorted(rs["kernels"].items(), key=lambda kv: -kv[1]["pct"])[:6]
        for k, v in top:
            print(f"{tag} {v['pct']:6.2f}%  {v['avg_us']:10.2f} us  x{v['calls']:4d}  {k[:100]}")
        print(tag, json.dumps(rs["mix_pmc"], indent=1))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--ranks"]
    main(args[0], args[1], ranks="--ranks" in sys.argv)
