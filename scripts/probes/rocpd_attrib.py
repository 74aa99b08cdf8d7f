"""Attribute blit kernels (copyBuffer / fillBuffer) of a rocprofv3 run to the HIP API calls that
issued them, from the rocpd SQLite database (ROCm 7):

    python scripts/probes/rocpd_attrib.py gpurun_out/<dir>/<run>_results.db

Prints the database's views and their columns first (the schema differs between ROCm releases),
then, per kernel name containing 'rocclr', the API calls sharing its correlation id with counts.
"""

import sqlite3
import sys
from collections import Counter


def cols(cur, name):
    return [r[1] for r in cur.execute(f"pragma table_info('{name}')")]


def main() -> None:
    db = sqlite3.connect(sys.argv[1])
    cur = db.cursor()
    objs = list(cur.execute("select type, name from sqlite_master where type in ('table','view') order by type, name"))
    for t, n in objs:
        if n.startswith("sqlite_"):
            continue
        print(f"{t:5s} {n}: {', '.join(cols(cur, n))[:300]}")
    names = {n for _, n in objs}
    if "kernels" not in names:
        return
    kc = cols(cur, "kernels")
    corr_k = next((c for c in ("correlation_id", "corr_id", "cid") if c in kc), None)
    api_view = next((v for v in ("regions", "region", "api", "hip_api", "regions_and_samples") if v in names), None)
    print("\nkernel corr column:", corr_k, "api view:", api_view)
    if not corr_k or not api_view:
        return
    ac = cols(cur, api_view)
    corr_a = next((c for c in ("correlation_id", "corr_id", "cid") if c in ac), None)
    if not corr_a:
        return
    apis = {}
    for cid, name in cur.execute(f"select {corr_a}, name from {api_view}"):
        apis[cid] = name
    per = {}
    for kname, cid in cur.execute(f"select name, {corr_k} from kernels"):
        if "rocclr" in kname or "Fill" in kname:
            per.setdefault(kname, Counter())[apis.get(cid, "?")] += 1
    for kname, cnt in per.items():
        print(f"\n{kname[:80]} ({sum(cnt.values())}):")
        for api, n in cnt.most_common(12):
            print(f"   {n:6d}  {api}")


if __name__ == "__main__":
    main()
