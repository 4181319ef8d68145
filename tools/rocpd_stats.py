#!/usr/bin/env python3
"""Per-kernel summary (the rocprofv3 --stats table) from a rocprofv3 rocpd
SQLite database, for committing under profiles/.

    python tools/rocpd_stats.py gpurun_out/<tag>/prof/run_results.db > profiles/<name>.csv
"""

import csv
import sqlite3
import statistics
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute("select name, duration from kernels").fetchall()
    by = {}
    for name, dur in rows:
        by.setdefault(name, []).append(dur)
    total = sum(sum(v) for v in by.values())
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDev"])
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), round(100.0 * sum(v) / total, 2),
                    min(v), max(v), statistics.pstdev(v)])


if __name__ == "__main__":
    main(sys.argv[1])
