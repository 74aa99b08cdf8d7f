"""Kernel statistics (CSV, like rocprofv3 --stats) from a rocprofv3 SQLite output database.

    python scripts/tools/rocpd_stats.py gpurun_out/<dir>/prof/run_results.db > profiles/<dir>/kernel_stats.csv
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main(path: str) -> None:
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = defaultdict(list)
    for name, s, e in rows:
        agg[name].append(e - s)
    total = sum(sum(v) for v in agg.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / total, 2), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
