"""GPU idle time between kernels in a rocprofv3 kernel trace (steady-state rounds)."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t_first = int(rows[len(rows)//3]["Start_Timestamp"]); t_last = int(rows[-1]["End_Timestamp"])
busy_end = None; idle = 0; big = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t_first: continue
    if busy_end is not None and s > busy_end:
        g = s - busy_end; idle += g
        if g > 20000: big.append((g / 1e3, prev_name[:30], r["Kernel_Name"][:30]))
    busy_end = e if busy_end is None else max(busy_end, e); prev_name = r["Kernel_Name"]
span = t_last - t_first
print(f"span {span/1e6:.2f} ms, idle {idle/1e6:.2f} ms ({100*idle/span:.1f}%), gaps>20us: {len(big)}")
for g in sorted(big, reverse=True)[:10]: print("  %.1f us after %s before %s" % g)
