"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches)."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0][:40]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add((path, r["Dispatch_Id"]))
for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", kv[1].get("GRBM_GUI_ACTIVE", 0))):
    n = max(1, len(calls[k]) // max(1, len(sys.argv) - 1))
    line = f"{k:40s} n={n:4d} " + " ".join(f"{name}={v / n:.4g}" for name, v in sorted(c.items()))
    print(line)
    # derived
    d = {}
    if c.get("SQ_WAVE_CYCLES"):
        d["wait_any%"] = 100 * c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        d["wait_inst%"] = 100 * c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        d["active%"] = 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if c.get("SQ_INSTS_LDS"):
        d["lds_conflict_per_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
    if c.get("SQ_BUSY_CU_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES"):
        d["mfma_busy%"] = 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_BUSY_CU_CYCLES"]
    if c.get("TCC_HIT_sum") is not None and (c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)):
        d["l2_hit%"] = 100 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if d:
        print(" " * 42 + " ".join(f"{a}={b:.3g}" for a, b in d.items()))
