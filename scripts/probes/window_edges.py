"""Device idle at the edges of bench.py's timed window (rocprofv3 CSV: kernel + marker traces).

    python scripts/probes/window_edges.py <dir with *_kernel_trace.csv and *_marker_api_trace.csv>

The bench marks its clock start (after barrier + synchronize) and end with roctx ("bench:t0",
"bench:t1", MYFYP_ROCTX=1). Prints t0 -> first kernel start, last kernel end -> t1, and the busy span.
"""
import csv
import glob
import os
import sys


def main() -> None:
    d = sys.argv[1]
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    mf = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)[0]
    marks = {}
    with open(mf) as f:
        for r in csv.DictReader(f):
            name = r.get("Function") or r.get("Operation") or ""
            msg = r.get("Message", "") or name
            for key in ("bench:t0", "bench:t1"):
                if key in msg or key in name:
                    marks[key] = int(r["Start_Timestamp"])
    ks = []
    with open(kf) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    t0, t1 = marks["bench:t0"], marks["bench:t1"]
    inside = [k for k in ks if k[0] >= t0 and k[1] <= t1]
    first = min(inside, key=lambda k: k[0])
    last = max(inside, key=lambda k: k[1])
    print(f"window {(t1 - t0) / 1e3:.1f} us; t0 -> first kernel start {(first[0] - t0) / 1e3:.1f} us ({first[2]}); "
          f"last kernel end -> t1 {(t1 - last[1]) / 1e3:.1f} us ({last[2]}); kernels {len(inside)}")


if __name__ == "__main__":
    main()
