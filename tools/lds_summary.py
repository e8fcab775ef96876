"""Summarise tools/prof_lds.sh counter CSVs: per kernel, totals over its
dispatches and the bank-conflict share of LDS cycles."""
import collections
import csv
import json
import sys

out = {}
for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    rows = {}
    for k, c in agg.items():
        if "consensus" not in k and "rank" not in k and "bonds" not in k:
            continue
        idx = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        rows[k] = {"dispatches": len(disp[k]), **{n: v for n, v in sorted(c.items())},
                   "bank_conflict_frac_of_lds_cycles": (c.get("SQ_LDS_BANK_CONFLICT", 0.0) / idx) if idx else 0.0}
    out[path] = rows
print(json.dumps(out, indent=1))
