"""Writes simulation_results_b{β}.html for the four bond penalties — the
reference's scripts/charts_table_generator.py. The simulations run on the
MI355X engine (each (case, version) once, v1.api.generate_chart_table);
the charts render on the CPU with matplotlib."""

from __future__ import annotations

import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PKG = os.path.join(_ROOT, "yuma-simulation_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from yuma_simulation._internal.cases import cases  # noqa: E402
from yuma_simulation._internal.simulation_utils import SHEET_BOND_PENALTIES, sheet_yuma_versions  # noqa: E402
from yuma_simulation._internal.yumas import SimulationHyperparameters  # noqa: E402
from yuma_simulation.v1.api import generate_chart_table  # noqa: E402


def main(out_dir: str = ".") -> list[str]:
    written = []
    for bond_penalty in SHEET_BOND_PENALTIES:
        hyper = SimulationHyperparameters(bond_penalty=bond_penalty)
        table = generate_chart_table(cases, sheet_yuma_versions(), hyper, draggable_table=True)
        path = os.path.join(out_dir, f"simulation_results_b{bond_penalty}.html")
        with open(path, "w", encoding="utf-8") as f:
            f.write(table.data)
        print(f"HTML saved to {path}")
        written.append(path)
    return written


if __name__ == "__main__":
    main(*sys.argv[1:2])
