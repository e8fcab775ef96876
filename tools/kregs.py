"""Per-kernel register use of a built engine library: VGPRs, AGPRs, SGPRs and
spills from the gfx950 code object's metadata notes.
    python tools/kregs.py [lib.so] [name-filter ...]"""
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(lib):
    with tempfile.TemporaryDirectory() as t:
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={t}/fb", lib], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={t}/fb",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t}/co"], check=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f"{t}/co"], check=True,
                              capture_output=True, text=True).stdout


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else "yuma-simulation_amd/lib/libyuma_hip.so"
    filt = sys.argv[2:]
    txt = notes(lib)
    for blk in re.split(r"\n\s+- \.", txt):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m:
            continue
        name = subprocess.run(["c++filt"], input=m.group(1), capture_output=True, text=True).stdout.strip()
        if filt and not any(f in name for f in filt):
            continue
        g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
        print(f"v{g('vgpr_count'):>4} s{g('sgpr_count'):>4} vsp{g('vgpr_spill_count'):>4} "
              f"ssp{g('sgpr_spill_count'):>4} lds{g('group_segment_fixed_size'):>6}  {name[:160]}")


if __name__ == "__main__":
    main()
