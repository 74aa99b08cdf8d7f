"""Per-period device timeline of a rocprofv3 run (rocpd SQLite, ROCm 7): busy time, idle gaps and
the kernels of one steady-state period, where a period starts at each dispatch of a marker kernel.

    python scripts/probes/rocpd_timeline.py <run_results.db> <marker substring> [period index] [seq]

With a fourth argument ``seq`` it also lists the period's dispatches in start order: start and end
offsets from the period start (us), stream id and kernel.
"""

import sqlite3
import statistics
import sys
from collections import defaultdict


def main() -> None:
    db = sqlite3.connect(sys.argv[1])
    marker = sys.argv[2]
    rows = list(db.execute("select k.start, k.end, k.stream_id, s.kernel_name from rocpd_kernel_dispatch k "
                           "join rocpd_info_kernel_symbol s on k.kernel_id = s.id order by k.start"))
    marks = [i for i, r in enumerate(rows) if marker in r[3]]
    if len(marks) < 3:
        print("marker dispatches:", len(marks))
        return
    periods = [(rows[b][0] - rows[a][0]) / 1e3 for a, b in zip(marks, marks[1:])]
    print(f"{len(marks)} periods; median {statistics.median(periods):.1f} us, min {min(periods):.1f}, max {max(periods):.1f}")
    k = int(sys.argv[3]) if len(sys.argv) > 3 else len(marks) // 2
    a, b = marks[k], marks[k + 1]
    t0, t1 = rows[a][0], rows[b][0]
    per = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    end = t0
    gaps = 0.0
    for r in rows[a:b]:
        name = r[3].split("(")[0]
        per[name][0] += 1
        per[name][1] += (r[1] - r[0]) / 1e3
        if r[0] > end:
            gaps += (r[0] - end) / 1e3
        end = max(end, r[1])
    span = (t1 - t0) / 1e3
    busy = span - gaps
    print(f"period {k}: {span:.1f} us, device busy (any stream) {busy:.1f} us, idle {gaps:.1f} us, {b - a} dispatches")
    for name, (n, us) in sorted(per.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"  {us:9.1f} us  {n:4d}x  {name[:110]}")
    if len(sys.argv) > 4 and sys.argv[4] == "seq":
        for r in rows[a : b + 1]:
            print(f"  {(r[0] - t0) / 1e3:9.1f} {(r[1] - t0) / 1e3:9.1f}  s{r[2]}  {r[3].split('(')[0][:90]}")


if __name__ == "__main__":
    main()
