"""cProfile of the c5 sheet step on the GPU box (host side of the 504-run
dividend sheet: where its milliseconds go)."""
import cProfile
import os
import pstats
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
for _ in range(3):
    su.generate_total_dividends_tables(cases, v, hypers)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    su.generate_total_dividends_tables(cases, v, hypers)
torch.cuda.synchronize()
print("ms per sheet", (time.perf_counter() - t) / 10 * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    su.generate_total_dividends_tables(cases, v, hypers)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
