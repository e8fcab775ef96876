"""Where a kernel waits for all its vector-memory operations (s_waitcnt
vmcnt(0)) relative to its loops: disassembles a built engine library and
prints, per matching kernel, each vmcnt(0) with its loop depth and the next
instructions. A vmcnt(0) inside an epoch loop drains every prefetch in
flight (round 5: the rq4 record copy and a lane branch in the scans).
    python tools/waitcnt_map.py [lib.so] name-regex"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = sys.argv[1] if len(sys.argv) > 2 else os.path.join(ROOT, "yuma-simulation_amd", "lib", "libyuma_hip.so")
pat = re.compile(sys.argv[-1])
LLVM = "/opt/rocm/lib/llvm/bin"
with tempfile.TemporaryDirectory() as t:
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb", lib], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/fb",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/co"], check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f"{t}/co"],
                         capture_output=True, text=True, check=True).stdout
funcs = re.split(r"\n(?=[0-9a-f]+ <[^>]+>:\n)", dis)
for f in funcs:
    m = re.match(r"([0-9a-f]+) <([^>]+)>:", f)
    if not m:
        continue
    name = subprocess.run(["c++filt"], input=m.group(2), capture_output=True, text=True).stdout.strip()
    if not pat.search(name):
        continue
    ins = []
    for line in f.split("\n")[1:]:
        mm = re.match(r"\s+(\S.*?)\s*// ([0-9A-Fa-f]+):", line)
        if mm:
            ins.append((int(mm.group(2), 16), mm.group(1).strip()))
    addr = [a for a, _ in ins]
    loops = []  # (target, branch address) of backward branches
    for a, s in ins:
        if s.startswith(("s_cbranch", "s_branch")):
            parts = s.split()
            if len(parts) > 1 and parts[1].lstrip("-").isdigit():
                off = int(parts[1])
                off = off - 65536 if off > 32767 else off
                tgt = a + 4 + 4 * off
                if tgt <= a:
                    loops.append((tgt, a))
    print(f"== {name[:110]}  ({len(ins)} instructions, {len(loops)} back edges)")
    if os.environ.get("LOOPS"):
        for lo, hi in sorted(loops):
            print(f"   back edge {hi:x} -> {lo:x} ({(hi - lo) // 4} dwords)")
    for k, (a, s) in enumerate(ins):
        if "vmcnt(0)" in s:
            depth = sum(1 for lo, hi in loops if lo <= a <= hi)
            nxt = " | ".join(x for _, x in ins[k + 1:k + 3])
            print(f"  {a:x} loop depth {depth}: {nxt[:90]}")
