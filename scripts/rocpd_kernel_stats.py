"""Per-kernel summary of a rocprofv3 --kernel-trace run whose output is the
rocpd SQLite database (rocprofv3's default format on this image), in the
columns of rocprofv3's kernel_stats.csv:
    python scripts/rocpd_kernel_stats.py gpurun_out/r04/prof/run_results.db > profiles/r04/kernel_stats.csv"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                  "from kernels group by name order by sum(duration) desc").fetchall()
total = sum(r[2] for r in rows) or 1
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for name, n, tot, avg, mn, mx in rows:
    w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 4), mn, mx])
