"""How much of each matching kernel's run time overlaps other kernels (rocprofv3 SQLite output).

    python scripts/tools/kernel_overlap.py <run_results.db> <substring> [<substring> ...]

For every kernel whose name contains a substring: calls, total ns, ns during which some OTHER
kernel (not matching) was running on the device, and the queues/streams involved.
"""
import json
import sqlite3
import sys
from collections import defaultdict


def main(db: str, pats) -> None:
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    extra = [x for x in ("stream_id", "queue_id") if x in cols]
    rows = c.execute(f"select {name}, start, end{''.join(', ' + x for x in extra)} from kernels order by start").fetchall()
    mine = [r for r in rows if any(p in r[0] for p in pats)]
    other = [r for r in rows if not any(p in r[0] for p in pats)]
    res = defaultdict(lambda: {"calls": 0, "ns": 0, "overlapped_ns": 0, "streams": set(), "overlapping_kernels": defaultdict(int)})
    j0 = 0
    for r in mine:
        n, s, e = r[0], r[1], r[2]
        d = res[n]
        d["calls"] += 1
        d["ns"] += e - s
        if extra:
            d["streams"].add(tuple(r[3:]))
        while j0 < len(other) and other[j0][2] < s - 10**9:
            j0 += 1
        ivs = []
        for o in other[j0:]:
            if o[1] >= e:
                break
            lo, hi = max(s, o[1]), min(e, o[2])
            if hi > lo:
                ivs.append((lo, hi))
                d["overlapping_kernels"][o[0][:60]] += hi - lo
        ivs.sort()
        cov, cur_lo, cur_hi = 0, None, None
        for lo, hi in ivs:
            if cur_hi is None or lo > cur_hi:
                if cur_hi is not None:
                    cov += cur_hi - cur_lo
                cur_lo, cur_hi = lo, hi
            else:
                cur_hi = max(cur_hi, hi)
        if cur_hi is not None:
            cov += cur_hi - cur_lo
        d["overlapped_ns"] += cov
    for n, d in res.items():
        top = sorted(d["overlapping_kernels"].items(), key=lambda kv: -kv[1])[:5]
        print(json.dumps({"kernel": n[:90], "calls": d["calls"], "total_us": round(d["ns"] / 1e3, 1), "overlapped_us": round(d["overlapped_ns"] / 1e3, 1),
                          "overlap_frac": round(d["overlapped_ns"] / max(1, d["ns"]), 3), "streams_queues": sorted(map(str, d["streams"]))[:4],
                          "top_overlapping": {k: round(v / 1e3, 1) for k, v in top}}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
