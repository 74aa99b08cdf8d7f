"""Summarise a rocprofv3 kernel trace: per-kernel time, and the per-step span vs busy time of the
MLP engine's 3-kernel steps (launch gaps inside the graph)."""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
busy = defaultdict(float); cnt = defaultdict(int)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy[r["Kernel_Name"][:60]] += d; cnt[r["Kernel_Name"][:60]] += 1
for k, v in sorted(busy.items(), key=lambda x: -x[1])[:12]:
    print(f"{k:60s} n={cnt[k]:6d} total_ms={v/1e3:8.2f} avg_us={v/cnt[k]:7.2f}")
# step spans: fc1<true> start -> next fc1<true> start
starts = [r for r in rows if r["Kernel_Name"].startswith("void mlp_fc1_fwd<true>")]
spans = []
for a, b in zip(starts, starts[1:]):
    spans.append((int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3)
spans.sort()
if spans:
    print("step span us: p10 %.1f p50 %.1f p90 %.1f" % (spans[len(spans)//10], spans[len(spans)//2], spans[9*len(spans)//10]))
# gap analysis for consecutive kernels
gaps = defaultdict(list)
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if 0 <= g < 50:
        gaps[(a["Kernel_Name"][:25], b["Kernel_Name"][:25])].append(g)
for k, v in sorted(gaps.items(), key=lambda x: -len(x[1]))[:6]:
    v.sort(); print("gap", k, "n", len(v), "p50 %.2f us" % v[len(v)//2])
# round span: between consecutive eval kernels
ev = [r for r in rows if r["Kernel_Name"].startswith("void mlp_fc1_fwd<false>")]
es = [(int(b["Start_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3 for a, b in zip(ev, ev[1:])]
es.sort()
if es: print("round span (eval->eval) us: p50 %.1f min %.1f" % (es[len(es)//2], es[0]))
