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


def main(src, dst):
    stats = rows(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    kernels = {}
    for r in stats:
        name = pick(r, "Name", "KernelName")
        kernels[name] = {"calls": int(pick(r, "Calls")), "avg_us": float(pick(r, "AverageNs")) / 1e3,
                         "min_us": float(pick(r, "MinNs")) / 1e3, "max_us": float(pick(r, "MaxNs")) / 1e3,
                         "pct": float(pick(r, "Percentage"))}
    fetch = counter_per_kernel(os.path.join(src, "fetch"), "FETCH_SIZE")
    write = counter_per_kernel(os.path.join(src, "write"), "WRITE_SIZE")
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
    out = {"source": src, "kernels": kernels, "mix_pmc": mix, "pmc_all": allk,
           "note": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> bytes x1024"}
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    top = sorted(kernels.items(), key=lambda kv: -kv[1]["pct"])[:6]
    for k, v in top:
        print(f"{v['pct']:6.2f}%  {v['avg_us']:10.2f} us  x{v['calls']:4d}  {k[:100]}")
    print(json.dumps(mix, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
