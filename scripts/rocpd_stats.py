"""Dump the per-kernel summary (calls, total/avg ns, %) of a rocprofv3 rocpd database as CSV.

    python scripts/rocpd_stats.py gpurun_out/<tag>/prof/run_results.db > profiles/<name>.csv
"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
for name, calls, total, avg, pct in db.execute("select name,total_calls,total_duration,average,percentage from top_kernels"):
    # rocpd stores durations in us in this view
    w.writerow([name, calls, int(round(total * 1e3)), int(round(avg * 1e3)), round(pct, 3)])
