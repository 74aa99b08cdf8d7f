"""Per-kernel counter table from rocprofv3 --pmc CSV outputs (counter_collection.csv files).

    python scripts/tools/pmc_table.py a_counter_collection.csv b_counter_collection.csv > table.md

Kernels are grouped by name up to the argument list; counters are summed over dispatches. Derived
columns: VALU / MFMA, LDS bank conflicts per LDS instruction, wait share (SQ_WAIT_INST_ANY /
SQ_BUSY_CYCLES-normalised wave cycles) when the counters are present.
"""
import csv
import sys
from collections import defaultdict


def main(paths):
    tot = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((p, r["Dispatch_Id"]))
    print("| kernel | dispatches | VALU / MFMA | LDS insts / MFMA | LDS bank conflicts per LDS inst | VMEM rd+wr / MFMA | wait-any / active |")
    print("|---|---|---|---|---|---|---|")
    rows = sorted(tot.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0.0))
    for k, c in rows:
        mf = c.get("SQ_INSTS_MFMA", 0.0)
        f = lambda num, den: f"{num / den:.2f}" if den else "—"
        ndisp = len({d for (p, d) in calls[k] if p == paths[0]}) if paths else 0
        print(f"| `{k}` | {ndisp} | {f(c.get('SQ_INSTS_VALU', 0.0), mf)} | {f(c.get('SQ_INSTS_LDS', 0.0), mf)} | "
              f"{f(c.get('SQ_LDS_BANK_CONFLICT', 0.0), c.get('SQ_INSTS_LDS', 0.0))} | "
              f"{f(c.get('SQ_INSTS_VMEM_RD', 0.0) + c.get('SQ_INSTS_VMEM_WR', 0.0), mf)} | "
              f"{f(c.get('SQ_WAIT_ANY', 0.0), c.get('SQ_WAIT_ANY', 0.0) + c.get('SQ_ACTIVE_INST_ANY', 0.0))} |")


if __name__ == "__main__":
    main(sys.argv[1:])
