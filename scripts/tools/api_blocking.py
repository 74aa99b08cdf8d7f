"""Host-blocking HIP calls and GPU idle gaps in a rocprofv3 csv trace (--hip-trace --kernel-trace
--memory-copy-trace). Usage: api_blocking.py <trace dir>. Looks at the last half of the run (steady
state): per HIP function count / total / max time per thread, the calls that took > 50 us, and the
GPU's idle time between kernels with what preceded each large gap."""
import csv
import glob
import sys
from collections import defaultdict


def load(pattern):
    files = glob.glob(pattern, recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    return rows


d = sys.argv[1]
api = load(f"{d}/**/*hip_api_trace.csv")
kern = sorted(load(f"{d}/**/*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
copies = load(f"{d}/**/*memory_copy_trace.csv")
if not kern:
    sys.exit("no kernel trace found under " + d)
t_mid = int(kern[len(kern) // 2]["Start_Timestamp"])
t_end = int(kern[-1]["End_Timestamp"])
span = (t_end - t_mid) / 1e3
print(f"steady-state window: {span / 1e3:.2f} ms (last half of the kernels)")

stat = defaultdict(lambda: [0, 0.0, 0.0])
slow = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t_mid or s > t_end:
        continue
    k = (r["Function"], r.get("Thread_Id", "?"))
    dur = (e - s) / 1e3
    st = stat[k]
    st[0] += 1
    st[1] += dur
    st[2] = max(st[2], dur)
    if dur > 50:
        slow.append((dur, r["Function"], r.get("Thread_Id", "?"), (s - t_mid) / 1e3))
print("\nHIP API in the window (function, thread): calls, total us, max us")
for (fn, th), (n, tot, mx) in sorted(stat.items(), key=lambda x: -x[1][1])[:25]:
    print(f"  {fn:40s} tid {th:>8s} n={n:6d} total={tot:10.1f} max={mx:8.1f}")
print(f"\ncalls > 50 us: {len(slow)}")
for dur, fn, th, at in sorted(slow, reverse=True)[:25]:
    print(f"  {dur:8.1f} us {fn} tid {th} at +{at:.1f} us")

busy_end = None
idle = 0.0
gaps = []
prev = None
for r in kern:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t_mid:
        continue
    if busy_end is not None and s > busy_end:
        g = (s - busy_end) / 1e3
        idle += g
        gaps.append((g, prev, r["Kernel_Name"][:40]))
    busy_end = e if busy_end is None else max(busy_end, e)
    prev = r["Kernel_Name"][:40]
print(f"\nGPU idle between kernels: {idle:.1f} us of {span:.1f} us ({100 * idle / max(span, 1e-9):.1f}%)")
by = defaultdict(list)
for g, a, b in gaps:
    by[(a, b)].append(g)
for (a, b), v in sorted(by.items(), key=lambda x: -sum(x[1]))[:12]:
    v.sort()
    print(f"  n={len(v):4d} total={sum(v):9.1f} p50={v[len(v) // 2]:7.1f} us  {a}  ->  {b}")
nc = [c for c in copies if int(c["Start_Timestamp"]) >= t_mid]
print(f"\nmemory copies in the window: {len(nc)}")
kinds = defaultdict(int)
for c in nc:
    kinds[c.get("Direction", "?")] += 1
print("  " + ", ".join(f"{k}: {v}" for k, v in kinds.items()))
