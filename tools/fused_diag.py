"""Diagnostics for the fused phase-1 kernel (not part of the product): per
phase device time at c2 and the number of hand-off sweeps that had to poll."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "yuma-simulation_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from yuma_simulation._internal import engine, synth  # noqa: E402
from yuma_simulation._internal.yumas import YumaConfig  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
V, M, N = 256, 4096, 1
dev = engine.device()
W = engine.synth_weights(0x5EED0002, E, N, V, M)
S = torch.from_numpy(synth.stakes(0x5EED0002, E, N, V)).to(dev)
prm = [engine.make_params(engine.VARIANT_YUMA3, YumaConfig())]
ws = torch.zeros(engine.workspace_bytes(engine.VARIANT_YUMA3, N, E, V, M, False), dtype=torch.uint8, device=dev)
engine.set_path(engine.PATH_FUSED if os.environ.get("FUSED", "1") == "1" else engine.PATH_MULTIPASS)
for rep in range(3):
    buf = [0.0] * len(engine.PHASES)
    engine.run(engine.VARIANT_YUMA3, prm, W, S, want_hist=True, workspace=ws, phase_ms=buf)
    torch.cuda.synchronize()
    print({k: round(v, 3) for k, v in zip(engine.PHASES, buf) if v}, engine.workspace_counters(ws), flush=True)
