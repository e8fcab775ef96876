"""Per-kernel means of one rocprofv3 SQ pass (tools/prof_r04.sh sq*): counts per
dispatch, the VALU issue fraction and the effective clock.

    python tools/sq_summary.py gpurun_out/prof_sqc3 [--skip 2] > profiles/r04/sq_c3.txt

VALU roofline (MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2
cycles on its SIMD; 256 CUs x 4 SIMDs): valu_frac = SQ_INSTS_VALU x 2 /
(1024 x clock x kernel time). Clock: GRBM_GUI_ACTIVE / 8 (summed over the 8
XCDs) / kernel time (the guide's DVFS item), and the 2.4 GHz peak."""
import argparse
import csv
import glob
import json
import os
import re
import statistics
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--skip", type=int, default=0, help="first dispatches of each kernel to drop")
ap.add_argument("--json", default=None, help="append a record to this sq_valu.json (bench.py load_sq)")
ap.add_argument("--workload", default=None, help='JSON of the bench workload key, e.g. {"V": 256, ...}')
ap.add_argument("--commit", default=None)
ap.add_argument("--build-id", default=None, help="yuma_build_id of the library (default: from the bench log)")
a = ap.parse_args()
if a.build_id is None:
    for log in (os.path.join(a.dir, "run.log"), a.dir.rstrip("/") + ".log"):
        if os.path.exists(log):
            for line in reversed(open(log).read().splitlines()):
                if line.startswith("{") and "engine_build_id" in line:
                    a.build_id = json.loads(line)["engine_build_id"]
                    break
        if a.build_id:
            break
files = glob.glob(os.path.join(a.dir, "**", "*counter_collection*.csv"), recursive=True)
if not files:
    raise SystemExit(f"no counter_collection csv under {a.dir}")
vals = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
dur = {}
for f in files:
    for r in csv.DictReader(open(f)):
        m = re.search(r"\b(k_[A-Za-z0-9_]+)", r.get("Kernel_Name", ""))
        if not m:
            continue
        key = (m.group(1), int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
        vals[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
per = defaultdict(list)
for (k, d), c in sorted(vals.items(), key=lambda kv: kv[0][1]):
    per[k].append((d, c))
out = {}
for k, lst in per.items():
    lst = lst[a.skip:] if len(lst) > a.skip else lst
    names = sorted({n for _, c in lst for n in c})
    mean = {n: statistics.mean(c.get(n, 0.0) for _, c in lst) for n in names}
    t = [dur[(k, d)] for d, _ in lst if (k, d) in dur]
    rec = {"dispatches": len(lst), "counters": mean}
    if t:
        ts = statistics.mean(t)
        rec["kernel_s"] = ts
        clk = mean.get("GRBM_GUI_ACTIVE", 0.0) / 8 / ts if ts > 0 else 0.0
        rec["clock_GHz"] = round(clk / 1e9, 3)
        if "SQ_INSTS_VALU" in mean and ts > 0:
            rec["valu_frac_peak_clock"] = round(mean["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * ts), 4)
            if clk > 0:
                rec["valu_frac_eff_clock"] = round(mean["SQ_INSTS_VALU"] * 2 / (1024 * clk * ts), 4)
        if "SQ_INSTS_SALU" in mean and ts > 0:
            # one SALU instruction per cycle per SIMD's scalar unit (shared by its waves)
            rec["salu_frac_peak_clock"] = round(mean["SQ_INSTS_SALU"] / (1024 * 2.4e9 * ts), 4)
    out[k] = rec
for k, rec in sorted(out.items(), key=lambda kv: -kv[1].get("kernel_s", 0)):
    print(k, json.dumps(rec))
if a.json:
    recs = []
    if os.path.exists(a.json):
        recs = json.load(open(a.json))
    wl = json.loads(a.workload) if a.workload else {}
    recs = [r for r in recs if r.get("workload") != wl]
    recs.append({"workload": wl, "commit": a.commit, "build_id": a.build_id, "source": a.dir, "kernels": out})
    json.dump(recs, open(a.json, "w"), indent=1)
