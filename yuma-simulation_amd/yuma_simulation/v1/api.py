"""Public API v1: the chart table (reference v1/api.py:24-132).

The reference re-runs run_simulation once per chart type for every
(case, version) (:48-67) — 4-5 identical simulations per cell. Here all
(case, version) simulations of the table are run up front as batched engine
calls (one per variant and shape) and the charts are rendered from those
results. Rendering stays on matplotlib (CPU).
"""

from __future__ import annotations

import pandas as pd

from yuma_simulation._internal.cases import BaseCase
from yuma_simulation._internal.charts_utils import (
    _plot_bonds,
    _plot_dividends,
    _plot_incentives,
    _plot_validator_server_weights,
)
from yuma_simulation._internal.simulation_utils import (
    SimulationRun,
    _generate_draggable_html_table,
    _generate_ipynb_table,
    run_simulations,
)
from yuma_simulation._internal.yumas import (
    SimulationHyperparameters,
    YumaConfig,
    YumaParams,
    YumaSimulationNames,
)

try:  # the reference returns IPython.display.HTML
    from IPython.display import HTML
except ImportError:  # pragma: no cover - IPython is optional here
    class HTML:  # minimal stand-in with the attributes callers use
        def __init__(self, data: str):
            self.data = data

        def _repr_html_(self) -> str:
            return self.data


def _full_case_name(case: BaseCase, version: str, config: YumaConfig) -> str:
    names = YumaSimulationNames()
    title = f"{case.name} - {version}"
    if version in (names.YUMA, names.YUMA_LIQUID, names.YUMA2):
        return f"{title} - beta={config.bond_penalty}"
    if version == names.YUMA4_LIQUID:
        return f"{title} [{config.alpha_low}, {config.alpha_high}]"
    return title


def generate_chart_table(
    cases: list[BaseCase],
    yuma_versions: list[tuple[str, YumaParams]],
    yuma_hyperparameters: SimulationHyperparameters,
    draggable_table: bool = False,
) -> HTML:
    table_data: dict[str, list[str]] = {version: [] for version, _ in yuma_versions}
    # The reference collects each row as {version: chart} (reference v1/api.py:34-36, 50-119), so
    # a version listed twice keeps one column, filled by its LAST entry
    # (that entry's params and title), at the position of its first.
    last_params = {version: params for version, params in yuma_versions}
    versions = [(version, last_params[version]) for version in table_data]
    configs = [YumaConfig(simulation=yuma_hyperparameters, yuma_params=p) for _, p in versions]
    runs = [SimulationRun(case, version, cfg) for case in cases for (version, _), cfg in zip(versions, configs)]
    results = run_simulations(runs)
    case_row_ranges = []
    row = 0
    k = 0
    for idx, case in enumerate(cases):
        chart_types = ["weights", "dividends", "bonds", "normalized_bonds"]
        if idx in (9, 10):
            chart_types.append("incentives")
        per_version = results[k:k + len(versions)]
        k += len(versions)
        start = row
        for chart_type in chart_types:
            for ((version, _), cfg), (dividends, bonds, incentives) in zip(zip(versions, configs), per_version):
                title = _full_case_name(case, version, cfg)
                if chart_type == "weights":
                    img = _plot_validator_server_weights(case.validators, case.weights_epochs, case.servers,
                                                         case.num_epochs, title, to_base64=True)
                elif chart_type == "dividends":
                    img = _plot_dividends(case.num_epochs, case.validators, dividends, title,
                                          case.base_validator, to_base64=True)
                elif chart_type in ("bonds", "normalized_bonds"):
                    img = _plot_bonds(case.num_epochs, case.validators, case.servers, bonds, title,
                                      to_base64=True, normalize=chart_type == "normalized_bonds")
                else:
                    img = _plot_incentives(case.servers, incentives, case.num_epochs, title, to_base64=True)
                table_data[version].append(img)
            row += 1
        case_row_ranges.append((start, row - 1, idx))
    summary = pd.DataFrame(table_data)
    make = _generate_draggable_html_table if draggable_table else _generate_ipynb_table
    return HTML(make(table_data, summary, case_row_ranges))
