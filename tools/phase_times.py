"""Per-phase device time (HIP events, yuma_run_profiled) of one engine
configuration on resident synthetic inputs — the A/B harness for kernel
variants (not part of the product).

    python tools/phase_times.py [--version "Yuma 3 (Rhef)"] [--liquid] [--reps 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "yuma-simulation_amd"), ROOT]
import torch  # noqa: E402

from yuma_simulation._internal import engine, synth  # noqa: E402
from yuma_simulation._internal.simulation_utils import resolve_version  # noqa: E402
from yuma_simulation._internal.yumas import YumaConfig, YumaParams  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--version", default="Yuma 3 (Rhef)")
ap.add_argument("--liquid", action="store_true")
ap.add_argument("--epochs", type=int, default=1000)
ap.add_argument("--V", type=int, default=256)
ap.add_argument("--M", type=int, default=4096)
ap.add_argument("--N", type=int, default=1)
ap.add_argument("--no-history", action="store_true")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--tag", default="")
a = ap.parse_args()
variant, _ = resolve_version(a.version)
E, V, M, N = a.epochs, a.V, a.M, a.N
dev = engine.device()
W = engine.synth_weights(0x5EED0002, E, N, V, M)
S = torch.from_numpy(synth.stakes(0x5EED0002, E, N, V)).to(dev)
prm = [engine.make_params(variant, YumaConfig(yuma_params=YumaParams(liquid_alpha=a.liquid)))] * N
ws = torch.empty(engine.workspace_bytes(variant, N, E, V, M, False), dtype=torch.uint8, device=dev)
out = {"B_hist": None if a.no_history else torch.empty(E, N, V, M, device=dev)}
best = None
for rep in range(a.reps + 1):
    buf = [0.0] * len(engine.PHASES)
    engine.run(variant, prm, W, S, want_hist=not a.no_history, workspace=ws, phase_ms=buf, out=out)
    if rep == 0:
        continue  # warm-up
    tot = sum(buf)
    if best is None or tot < best[0]:
        best = (tot, buf)
print(a.tag, a.version, "liquid" if a.liquid else "", f"total {best[0]:.3f} ms",
      {k: round(v, 3) for k, v in zip(engine.PHASES, best[1]) if v}, flush=True)
