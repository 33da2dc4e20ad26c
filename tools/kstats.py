"""Print a rocprofv3 kernel_stats.csv as name / calls / avg us / total ms / %."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(r["Name"][:80].ljust(82), r["Calls"].rjust(5), "%9.1f" % (float(r["AverageNs"]) / 1e3),
          "%9.3f" % (float(r["TotalDurationNs"]) / 1e6), r["Percentage"][:5])
