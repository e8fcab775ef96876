"""Timing-only builds of the engine with parts of the consensus search cut
out (results are wrong; never used for parity): where k_consensus_w's time
goes at c2. Writes ablib/diag_<name>.so from patched copies of the product
source; time them with tools/ab_lib.sh.

    python tools/diag_consensus.py   # then: bash tools/ab_lib.sh ablib/diag_*.so
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

SRC = open(g.SRC).read()
ATOMIC = "atomicAdd(cb + (k < w ? k : w), su[i]);"
HIST_ON = "hist = bracket && ut >= 0;  // slice-uniform"
PATCHES = {
    # histogram bins written by plain LDS stores instead of integer atomics
    "nortn": [(ATOMIC, "cb[k < w ? k : w] = su[i];")],
    # no histogram finish and no bisection: load, divide, prerank, bracket
    "bracket": [(HIST_ON, "hist = false; lim = 1 << 30;")],
}

os.makedirs(os.path.join(ROOT, "ablib"), exist_ok=True)
for name, reps in PATCHES.items():
    s = SRC
    for a, b in reps:
        assert s.count(a) == 1, (name, a)
        s = s.replace(a, b)
    src = f"/tmp/diag_{name}.hip"
    open(src, "w").write(s)
    out = os.path.join(ROOT, "ablib", f"diag_{name}.so")
    cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *g.HIPCC_FLAGS,
           "-I", os.path.join(ROOT, "include"), "-o", out, src]
    subprocess.run(cmd, check=True)
    print(out)
