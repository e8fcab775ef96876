"""Steady-state per-kernel durations from a rocprofv3 kernel trace: all
launches (what --stats averages) and the launches after the first `skip`
(an idle MI355X ramps its clocks over the first few steps).

    python tools/trace_stats.py profiles/r03/c2y3/kernel_trace.csv [--skip 6]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--skip", type=int, default=6)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
d = defaultdict(list)
for r in rows:
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
    if m:
        d[m.group(1)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(f"{'kernel':16s} {'calls':>5s} {'mean_all':>9s} {'mean_steady':>11s} {'median':>8s} {'min':>8s}  (ms; steady = after the first {a.skip})")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    st = v[a.skip:] if len(v) > a.skip else v
    print(f"{k:16s} {len(v):5d} {statistics.mean(v):9.4f} {statistics.mean(st):11.4f} {statistics.median(v):8.4f} {min(v):8.4f}")
