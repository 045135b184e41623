"""Kernel summary (name, calls, total / average / min / max ns) from a
rocprofv3 rocpd SQLite database (the default output of rocprofv3 7.x), in the
column layout of rocprofv3's kernel_stats.csv.  usage: rocpd_summary.py DB [CSV]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                  "from kernels group by name order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
for n, c, s, a, mn, mx in rows:
    out.append([n, c, s, round(a, 1), round(100.0 * s / tot, 2), mn, mx])
if len(sys.argv) > 2:
    with open(sys.argv[2], "w", newline="") as f:
        csv.writer(f).writerows(out)
for r in out[:25]:
    print(*r, sep=" | ")
