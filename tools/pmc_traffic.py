"""Turn rocprofv3 PMC passes into per-kernel HBM bytes (profiles/r03/pmc_traffic.json,
one record per bench workload; bench.py reads roofline.traffic from it).

Two separate counter passes of the same bench command (MI355X_MICROARCH.md
§HBM: FETCH_SIZE and WRITE_SIZE do not fit one pass):

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d gpurun_out/pmc_fetch -o fetch -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d gpurun_out/pmc_write -o write -- python3 bench.py ...

Corrections applied (gfx950, per the guide): FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled (the dominant loads here are float4 streams);
WRITE_SIZE is exact for 16 B/lane streaming stores. The Infinity Cache is
counted, not excluded.

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write \
        --epochs 1000 --scenarios 1 --V 256 --M 4096 --version "Yuma 3 (Rhef)" --history
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics
from collections import defaultdict

KERNEL_RE = re.compile(r"\b(k_[A-Za-z0-9_]+)")


def counters(directory: str, name: str) -> dict[str, list[float]]:
    """kernel name -> list of per-dispatch counter values (KiB)."""
    files = glob.glob(os.path.join(directory, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {directory}")
    per_dispatch: dict[tuple, float] = defaultdict(float)
    kname: dict[tuple, str] = {}
    for path in files:
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != name:
                    continue
                key = (path, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per_dispatch[key] += float(row["Counter_Value"])
                kname[key] = row.get("Kernel_Name", "")
    out: dict[str, list[float]] = defaultdict(list)
    for key, v in per_dispatch.items():
        m = KERNEL_RE.search(kname[key])
        if m and m.group(1) != "k_synth":
            out[m.group(1)].append(v)
    return out


def bench_build_id(directory: str) -> str | None:
    """engine_build_id of the bench line a pass ran (its log: <dir>.log or
    <dir>/run.log, last JSON line)."""
    for log in (directory.rstrip("/") + ".log", os.path.join(directory, "run.log")):
        if os.path.exists(log):
            for line in reversed(open(log).read().splitlines()):
                if line.startswith("{"):
                    try:
                        return json.loads(line).get("engine_build_id")
                    except ValueError:
                        continue
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--epochs", type=int, required=True)
    ap.add_argument("--scenarios", type=int, default=1)
    ap.add_argument("--V", type=int, default=256)
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--version", default="Yuma 3 (Rhef)")
    ap.add_argument("--history", action="store_true")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "r04",
                                                  "pmc_traffic.json"))
    ap.add_argument("--commit", default=None, help="git commit of the library the passes ran (ADVICE r3)")
    ap.add_argument("--launches", type=int, default=1, help="launches of each kernel per bench step")
    ap.add_argument("--build-id", default=None, help="yuma_build_id of the library (default: from the bench logs)")
    a = ap.parse_args()
    bid = a.build_id
    if bid is None:
        ids = {bench_build_id(a.fetch_dir), bench_build_id(a.write_dir)}
        if len(ids) != 1 or None in ids:
            raise SystemExit(f"the FETCH and WRITE passes ran different / unknown builds: {ids}")
        bid = ids.pop()
    fetch = counters(a.fetch_dir, "FETCH_SIZE")
    write = counters(a.write_dir, "WRITE_SIZE")
    units = a.epochs * a.scenarios
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch[k]) if fetch.get(k) else 0.0
        w = statistics.median(write[k]) if write.get(k) else 0.0
        read_b = 2.0 * f * 1024.0   # gfx950: FETCH_SIZE = half of wide streaming reads
        write_b = w * 1024.0
        kernels[k] = {
            "fetch_size_kib_raw": f,
            "write_size_kib": w,
            "hbm_read_bytes_per_launch": read_b,
            "hbm_write_bytes_per_launch": write_b,
            "hbm_bytes_per_launch": read_b + write_b,
            "hbm_bytes_per_scenario_epoch": (read_b + write_b) * a.launches / units,
            "dispatches": [len(fetch.get(k, [])), len(write.get(k, []))],
        }
    rec = {
        "workload": {"V": a.V, "M": a.M, "epochs": a.epochs, "scenarios_per_gpu": a.scenarios,
                     "version": a.version, "bond_history": bool(a.history)},
        "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), KiB -> bytes; WRITE_SIZE as is",
        "commit": a.commit,
        "build_id": bid,
        "step_hbm_bytes": sum(v["hbm_bytes_per_launch"] for v in kernels.values()) * a.launches,
        "kernels": kernels,
    }
    recs = []
    if os.path.exists(a.out):
        with open(a.out) as f:
            recs = [r for r in json.load(f) if r.get("workload") != rec["workload"]]
    recs.append(rec)
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(recs, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
