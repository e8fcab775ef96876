"""Writes total_dividends_b{β}.csv for the four bond penalties — the
reference's scripts/total_dividends_sheet_generator.py (same files, same
text), with every run of all four sheets batched on the MI355X engine
(generate_total_dividends_tables)."""

from __future__ import annotations

import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PKG = os.path.join(_ROOT, "yuma-simulation_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from yuma_simulation._internal.cases import cases  # noqa: E402
from yuma_simulation._internal.simulation_utils import (  # noqa: E402
    SHEET_BOND_PENALTIES,
    generate_total_dividends_tables,
    sheet_yuma_versions,
)
from yuma_simulation._internal.yumas import SimulationHyperparameters  # noqa: E402


def main(out_dir: str = ".") -> list[str]:
    hypers = [SimulationHyperparameters(bond_penalty=b) for b in SHEET_BOND_PENALTIES]
    print(f"Generating total dividends tables for bond_penalty in {list(SHEET_BOND_PENALTIES)}.")
    frames = generate_total_dividends_tables(cases, sheet_yuma_versions(), hypers)
    written = []
    for bond_penalty, df in zip(SHEET_BOND_PENALTIES, frames):
        if df.isnull().values.any():
            print(f"CSV for bond_penalty={bond_penalty} contains missing values. Please check the simulation data.")
        else:
            print(f"No missing values detected in the CSV data for bond_penalty={bond_penalty}.")
        path = os.path.join(out_dir, f"total_dividends_b{bond_penalty}.csv")
        df.to_csv(path, index=False, float_format="%.6f")
        print(f"CSV file {path} has been created successfully.")
        written.append(path)
    return written


if __name__ == "__main__":
    main(*sys.argv[1:2])
