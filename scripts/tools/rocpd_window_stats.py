"""Kernel statistics over a time window of a rocprofv3 trace (tuner / warm-up dispatches out).

    python scripts/tools/rocpd_window_stats.py <run_results.db | run_kernel_trace.csv> <name substring> <n>  > stats.csv

The window starts at the n-th dispatch (1-based) of a kernel whose name contains the substring
(e.g. the first optimizer step of the first timed round) and runs to the end of the trace; n = 0
starts it at the middle dispatch of that kernel (the second half of the run)."""
import csv
import sqlite3
import sys
from collections import defaultdict


def load(path: str):
    if path.endswith(".csv"):  # --kernel-trace CSV output (kernel_trace.csv)
        with open(path, newline="") as f:
            return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)]
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    return c.execute(f"select {name_col}, start, end from kernels").fetchall()


def main(path: str, marker: str, nth: int) -> None:
    rows = sorted(load(path), key=lambda r: r[1])
    hits = [r for r in rows if marker in r[0]]
    if nth == 0 and hits:
        nth = len(hits) // 2 + 1
    t0 = hits[nth - 1][1] if 0 < nth <= len(hits) else rows[0][1]
    agg = defaultdict(list)
    for name, s, e in rows:
        if s >= t0:
            agg[name].append(e - s)
    total = sum(sum(v) for v in agg.values()) or 1
    span = max(e for _, s, e in rows if s >= t0) - t0
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / total, 2), min(v), max(v)])
    print(f"# window from dispatch {nth} of '{marker}': span {span / 1e6:.3f} ms, kernel time {total / 1e6:.3f} ms", file=sys.stderr)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
