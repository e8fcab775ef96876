"""Split of the c5 sheet step on the GPU box: the batched engine runs with
their per-run dividend totals (_run_simulations, totals=True) against the four
sheet frames built from them (_sheet_frame_totals)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuma-simulation_amd")]
import torch  # noqa: E402

from yuma_simulation._internal import simulation_utils as su  # noqa: E402
from yuma_simulation._internal.cases import cases  # noqa: E402
from yuma_simulation._internal.yumas import SimulationHyperparameters  # noqa: E402

hypers = [SimulationHyperparameters(bond_penalty=b) for b in su.SHEET_BOND_PENALTIES]
v = su.sheet_yuma_versions()
per = [su._sheet_runs(cases, v, h) for h in hypers]
flat_runs = [r for runs in per for r in runs]
for _ in range(3):
    su.generate_total_dividends_tables(cases, v, hypers)
torch.cuda.synchronize()
R = 20
t = time.perf_counter()
for _ in range(R):
    su.generate_total_dividends_tables(cases, v, hypers)
torch.cuda.synchronize()
whole = (time.perf_counter() - t) / R * 1e3
t = time.perf_counter()
for _ in range(R):
    with su._no_cyclic_gc():
        flat = [d for d, _, _ in su._run_simulations(flat_runs, False, False, totals=True)]
torch.cuda.synchronize()
runs_ms = (time.perf_counter() - t) / R * 1e3
t = time.perf_counter()
for _ in range(R):
    k = 0
    for runs in per:
        su._sheet_frame_totals(cases, v, flat[k:k + len(runs)])
        k += len(runs)
frames_ms = (time.perf_counter() - t) / R * 1e3
print(f"sheet {whole:.3f} ms = runs {runs_ms:.3f} + frames {frames_ms:.3f} (+ run/frame setup)")
