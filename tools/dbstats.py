"""Per-kernel average / count from a rocprofv3 SQLite output (prof_results.db): the `kernels`
view, last N dispatches of each kernel skipped = 0.  Usage: dbstats.py <db> [min_calls]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, count(*), avg(end - start), min(end - start) from kernels group by {name} "
                 f"order by sum(end - start) desc").fetchall()
for n, k, a, m in rows:
    if k >= int(sys.argv[2]) if len(sys.argv) > 2 else True:
        print(f"{n[:70]:72s} {k:5d} avg {a / 1e3:8.1f} us  min {m / 1e3:8.1f}")
