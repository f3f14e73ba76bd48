"""Kernel stats CSV (name, calls, total_us, avg_us, pct) from a rocprofv3 rocpd database."""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
cur = sqlite3.connect(db).execute(
    "select name, total_calls, total_duration, average, percentage from top_kernels")
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for r in cur:
        w.writerow(r)
print(open(out).read())
