"""Summarise a rocprofv3 run database (rocpd SQLite, ROCm 7) into per-kernel statistics.

    python scripts/probes/rocpd_summary.py gpurun_out/<dir>/run_results.db [out.csv]

Prints the top kernels (calls, total / mean µs, share of GPU time) and per-stream totals, and
writes the full table as CSV when an output path is given.
"""

import csv
import sqlite3
import sys


def main() -> None:
    db = sqlite3.connect(sys.argv[1])
    cur = db.cursor()
    rows = list(cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    print(f"{'kernel':90s} {'calls':>7s} {'total_us':>10s} {'mean_us':>9s} {'%':>6s}")
    for name, calls, tot, avg, pct in rows[:25]:
        print(f"{name[:90]:90s} {calls:7d} {tot / 1e3:10.1f} {avg / 1e3:9.2f} {pct:6.2f}")
    print("\nper stream (kernels, total us):")
    for sid, n, tot in cur.execute("select stream_id, count(*), sum(duration) from kernels group by stream_id order by 3 desc"):
        print(f"  stream {sid}: {n} kernels, {tot / 1e3:.1f} us")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["name", "calls", "total_ns", "mean_ns", "percent"])
            w.writerows(rows)


if __name__ == "__main__":
    main()
