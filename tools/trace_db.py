"""Per-kernel duration summary of a rocprofv3 rocpd database (prof_results.db): name, calls, avg /
min / max us.  python tools/trace_db.py <db> [<db> ...]"""
import sqlite3
import sys

for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(duration)/1000.0, min(duration)/1000.0, max(duration)/1000.0 "
         "from kernels group by name order by sum(duration) desc limit 12")
    print("##", db)
    for n, k, a, lo, hi in c.execute(q).fetchall():
        print("  %-60s %5d avg %8.2f min %8.2f max %8.2f" % (n[:60], k, a, lo, hi))
