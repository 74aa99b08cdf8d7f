"""Memory copies and kernels that fall inside the probe windows (rocprofv3 SQLite output).

    python scripts/tools/copies_in_window.py gpurun_out/agg/run_results.db gpurun_out/device_agg_windows.json
"""
import json
import sqlite3
import sys
from collections import Counter


def _table(c, *names):
    have = {r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")}
    for n in names:
        if n in have:
            return n
    return None


def main(db: str, windows: str) -> None:
    c = sqlite3.connect(db)
    kt = _table(c, "kernels")
    mt = _table(c, "memory_copies", "memory_copy")
    kcols = [r[1] for r in c.execute(f"pragma table_info({kt})")]
    kname = "kernel_name" if "kernel_name" in kcols else "name"
    kernels = c.execute(f"select {kname}, start, end from {kt}").fetchall()
    copies = []
    if mt:
        mcols = [r[1] for r in c.execute(f"pragma table_info({mt})")]
        dcol = next((x for x in ("name", "kind", "direction") if x in mcols), None)
        scol = "size" if "size" in mcols else ("bytes" if "bytes" in mcols else None)
        copies = c.execute(f"select {dcol or 'null'}, {scol or 0}, start, end from {mt}").fetchall()
    for w in json.load(open(windows)):
        t0, t1 = w["window_ns"]
        ks = Counter(n for n, s, e in kernels if s >= t0 and e <= t1)
        cs = [(d, b) for d, b, s, e in copies if s >= t0 and e <= t1]
        print(json.dumps({"kind": w["kind"], "iters": w["iters"], "us_per_call": w["us_per_call"], "copies_in_window": len(cs),
                          "copy_bytes": sum(int(b or 0) for _, b in cs), "copy_kinds": dict(Counter(str(d) for d, _ in cs)),
                          "kernels_per_call": {k: round(v / w["iters"], 2) for k, v in ks.most_common()}}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
