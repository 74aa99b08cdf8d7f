"""Per-period device idle time of a rocprofv3 kernel trace (rocpd SQLite), where a period starts at
each dispatch of a marker kernel; prints the period / idle distribution and the dispatch sequence
of the slowest and of the median period (start, end offsets in us, stream, kernel).

    python scripts/probes/rocpd_periods.py <run_results.db> <marker substring>
"""
import sqlite3
import statistics
import sys


def main() -> None:
    db = sqlite3.connect(sys.argv[1])
    marker = sys.argv[2]
    rows = list(db.execute("select k.start, k.end, k.stream_id, s.kernel_name from rocpd_kernel_dispatch k "
                           "join rocpd_info_kernel_symbol s on k.kernel_id = s.id order by k.start"))
    marks = [i for i, r in enumerate(rows) if marker in r[3]]
    out = []
    for a, b in zip(marks, marks[1:]):
        t0, t1 = rows[a][0], rows[b][0]
        end, idle = t0, 0.0
        for r in rows[a:b]:
            if r[0] > end:
                idle += (r[0] - end) / 1e3
            end = max(end, r[1])
        out.append(((t1 - t0) / 1e3, idle, a, b))
    out = out[3:]  # warmup periods
    per = [p for p, _, _, _ in out]
    idl = [i for _, i, _, _ in out]
    q = lambda v, f: sorted(v)[int(f * (len(v) - 1))]
    print(f"{len(out)} periods: period p10 {q(per, .1):.1f} p50 {q(per, .5):.1f} p90 {q(per, .9):.1f} max {max(per):.1f} us; "
          f"device idle p10 {q(idl, .1):.1f} p50 {q(idl, .5):.1f} p90 {q(idl, .9):.1f} max {max(idl):.1f} us; mean period {statistics.mean(per):.1f}")
    for label, sel in (("median", sorted(out)[len(out) // 2]), ("slowest", max(out))):
        p, i, a, b = sel
        print(f"--- {label} period: {p:.1f} us, idle {i:.1f} us")
        t0 = rows[a][0]
        for r in rows[a:b]:
            print(f"  {(r[0] - t0) / 1e3:9.1f} {(r[1] - t0) / 1e3:9.1f}  s{r[2]}  {r[3].split('(')[0][:90]}")


main()
