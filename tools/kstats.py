"""VGPR / SGPR / spill / scratch counts per kernel of a built engine library
(code-object metadata; no GPU needed).
    python tools/kstats.py [lib.so] [name-regex]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "yuma-simulation_amd", "lib", "libyuma_hip.so")
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
LLVM = "/opt/rocm/lib/llvm/bin"
with tempfile.TemporaryDirectory() as t:
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb", lib], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/fb",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/co"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", f"{t}/co"], capture_output=True, text=True).stdout
for e in re.split(r"\n\s*- \.agpr_count", notes):
    m = re.search(r"\.name:\s+(\S+)", e)
    if not m or not pat.search(m.group(1)):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", e) or [None, "-"])[1]
    dem = subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()
    print(f"vgpr {g('vgpr_count'):>3} sgpr {g('sgpr_count'):>3} vspill {g('vgpr_spill_count'):>4} "
          f"sspill {g('sgpr_spill_count'):>4} scratch {g('private_segment_fixed_size'):>4} lds {g('group_segment_fixed_size'):>5}  {dem}")
