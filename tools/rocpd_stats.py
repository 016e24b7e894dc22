"""Per-kernel time summary from a rocprofv3 rocpd database (the default output of rocprofv3 on
ROCm 7): python3 tools/rocpd_stats.py DIR [--csv OUT]"""
import csv
import glob
import sqlite3
import sys

dbs = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)
rows = []
for f in dbs:
    c = sqlite3.connect(f)
    q = ("select name, count(*), avg(end-start), sum(end-start), min(end-start), max(end-start) "
         "from kernels group by name order by sum(end-start) desc")
    rows += [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in c.execute(q)]
for r in rows[:25]:
    print(f"{r[0][:72]:72s} {r[1]:5d} avg {r[2] / 1e3:9.1f} us  total {r[3] / 1e6:8.2f} ms")
if "--csv" in sys.argv:
    with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Name", "Calls", "AverageNs", "TotalDurationNs", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 1), r[3], r[4], r[5]])
