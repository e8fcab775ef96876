"""Copy the rocprofv3 passes of tools/prof.sh runs (gpurun_out/prof_TAG) into
profiles/rNN/TAG (kernel stats, the kernel trace, gzipped counter CSVs, the
steady-state per-kernel table) and record each workload's PMC traffic in
profiles/rNN/pmc_traffic.json (tools/pmc_traffic.py).

    python tools/collect_prof.py r05 c2y3 c2y4l c3 c4 v1 v2 v0"""
import gzip
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {  # tag: (epochs, scenarios, V, M, version, history)
    "c2y3": (1000, 1, 256, 4096, "Yuma 3 (Rhef)", True),
    "c2y4l": (1000, 1, 256, 4096, "Yuma 4 (Rhef+relative bonds) - liquid alpha on", True),
    "c3": (32, 512, 256, 4096, "Yuma 4 (Rhef+relative bonds)", False),
    "c4": (100, 1, 256, 65536, "Yuma 3 (Rhef)", False),
    "v1": (1000, 1, 256, 4096, "Yuma 1 (paper)", True),
    "v2": (1000, 1, 256, 4096, "Yuma 2 (Adrian-Fish)", True),
    "v0": (1000, 1, 256, 4096, "Yuma 0 (subtensor)", True),
}


def main():
    rnd, tags = sys.argv[1], sys.argv[2:]
    commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
    for tag in tags:
        src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
        dst = os.path.join(ROOT, "profiles", rnd, tag)
        os.makedirs(dst, exist_ok=True)
        shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
        shutil.copy(os.path.join(src, "trace", "run_kernel_trace.csv"), os.path.join(dst, "kernel_trace.csv"))
        for name, sub in (("pmc_fetch_size.csv.gz", "fetch"), ("pmc_write_size.csv.gz", "write")):
            with open(os.path.join(src, sub, f"{sub}_counter_collection.csv"), "rb") as f, \
                    gzip.open(os.path.join(dst, name), "wb") as g:
                g.write(f.read())
        steady = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_stats.py"),
                                 os.path.join(dst, "kernel_trace.csv")], capture_output=True, text=True,
                                check=True).stdout
        with open(os.path.join(dst, "steady_stats.txt"), "w") as f:
            f.write(steady)
        E, N, V, M, version, hist = WORKLOADS[tag]
        cmd = [sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), os.path.join(src, "fetch"),
               os.path.join(src, "write"), "--epochs", str(E), "--scenarios", str(N), "--V", str(V), "--M", str(M),
               "--version", version, "--out", os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json"),
               "--commit", commit]
        if hist:
            cmd.append("--history")
        subprocess.run(cmd, check=True, capture_output=True)
        print(tag, "->", os.path.relpath(dst, ROOT))
        print(steady)


if __name__ == "__main__":
    main()
