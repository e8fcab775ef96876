"""A/B builds of the engine from patched copies of the product source, so
the product file carries no build switches.

    python tools/ab_build.py NAME [NAME ...]    -> ablib/NAME.so
    python tools/ab_build.py --list

Patch sets live in tools/ab_patches.py: PATCHES[NAME] = [(old, new), ...];
every `old` must occur exactly once in yuma_engine.hip (or give a third
element, the expected count). "base" builds the unpatched source, "rev_<git rev>" that revision's source. Time the
libraries with tools/ab_lib.sh or tools/phase_times.py (YUMA_HIP_LIB=...).
Timing-only patches (results wrong by design) are named diag_*; they are
never run by the tests."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.dirname(os.path.abspath(__file__))]
import __graft_entry__ as g  # noqa: E402
from ab_patches import PATCHES  # noqa: E402


def patched(name: str) -> str:
    if name.startswith("rev_"):  # the product source of a git revision, unpatched
        rel = os.path.relpath(g.SRC, ROOT)
        return subprocess.run(["git", "-C", ROOT, "show", f"{name[4:]}:{rel}"], check=True,
                              capture_output=True, text=True).stdout
    s = open(g.SRC).read()
    for rep in PATCHES.get(name, []):
        old, new = rep[0], rep[1]
        want = rep[2] if len(rep) > 2 else 1
        n = s.count(old)
        if n != want:
            raise SystemExit(f"{name}: expected {want} occurrence(s) of {old[:60]!r}, found {n}")
        s = s.replace(old, new)
    return s


def build(name: str) -> str:
    if name != "base" and not name.startswith("rev_") and name not in PATCHES:
        raise SystemExit(f"unknown patch set {name}")
    os.makedirs(os.path.join(ROOT, "ablib"), exist_ok=True)
    src = os.path.join(os.path.dirname(g.SRC), f".ab_{name}.hip")  # next to the original: same includes
    with open(src, "w") as f:
        f.write(patched(name))
    out = os.path.join(ROOT, "ablib", f"{name}.so")
    bid = g.source_build_id(open(src).read())
    cmd = [os.environ.get("HIPCC", "/opt/rocm/bin/hipcc"), *g.HIPCC_FLAGS, "-w", f'-DYUMA_BUILD_ID="{bid}"',
           "-I", os.path.join(ROOT, "include"), "-o", out, src]
    try:
        subprocess.run(cmd, check=True)
    finally:
        os.remove(src)
    return out


if __name__ == "__main__":
    names = sys.argv[1:]
    if names == ["--list"]:
        print("\n".join(["base", *PATCHES]))
        raise SystemExit(0)
    with ThreadPoolExecutor(max_workers=min(4, len(names) or 1)) as ex:
        for out in ex.map(build, names):
            print(out)
