"""Epoch driver and dividend tables on the MI355X engine.

Drop-in for the reference's _internal/simulation_utils.py:
  * ``run_simulation`` (reference :26-112) keeps its signature and return
    value, but the per-epoch Python loop becomes ONE engine call over all
    epochs (engine.run): no host round trip between epochs, bond resets
    (:62-88) applied on the device, and the bond history produced in one
    buffer;
  * ``run_simulations`` batches many (case, version, config) runs of equal
    shape into one engine call per variant — the dividend sheet (reference
    :319-381) packs all its runs this way;
  * dividends per 1000 tao are derived from the engine's normalised dividends
    with the reference's own tensor ops and Python-double formula (:95-107).
"""

from __future__ import annotations

import gc
from contextlib import contextmanager

from collections import defaultdict
from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from yuma_simulation._internal import engine
from yuma_simulation._internal.cases import BaseCase
from yuma_simulation._internal.charts_utils import _calculate_total_dividends
from yuma_simulation._internal.yumas import (
    SimulationHyperparameters,
    YumaConfig,
    YumaParams,
    YumaSimulationNames,
)

_NAMES = YumaSimulationNames()

# version string -> (engine variant, bond-reset rule); reference dispatch :52-93
VERSION_TABLE = {
    _NAMES.YUMA: (engine.VARIANT_YUMA1, engine.RESET_NONE),
    _NAMES.YUMA_LIQUID: (engine.VARIANT_YUMA1, engine.RESET_NONE),
    _NAMES.YUMA2: (engine.VARIANT_YUMA2, engine.RESET_NONE),
    _NAMES.YUMA3: (engine.VARIANT_YUMA3, engine.RESET_NONE),
    _NAMES.YUMA31: (engine.VARIANT_YUMA3, engine.RESET_ALWAYS),
    _NAMES.YUMA32: (engine.VARIANT_YUMA3, engine.RESET_IF_ZERO_CONSENSUS),
    _NAMES.YUMA4: (engine.VARIANT_YUMA4, engine.RESET_IF_ZERO_CONSENSUS),
    _NAMES.YUMA4_LIQUID: (engine.VARIANT_YUMA4, engine.RESET_IF_ZERO_CONSENSUS),
    "Yuma 0 (subtensor)": (engine.VARIANT_RUST, engine.RESET_NONE),
}


def resolve_version(yuma_version: str) -> tuple[int, int]:
    try:
        return VERSION_TABLE[yuma_version]
    except (KeyError, TypeError):
        raise ValueError("Invalid Yuma function.") from None


@dataclass
class SimulationRun:
    case: BaseCase
    yuma_version: str
    yuma_config: YumaConfig


def _dividend_ratio(config: YumaConfig, S: torch.Tensor, Dn: torch.Tensor) -> np.ndarray:
    """Reference simulation_utils.py:48-49,95-107 on CPU tensors of any shape
    [..., V]: the same elementwise torch ops (so the same fp32 roundings; a GPU
    `x / 1000.0` would be a reciprocal multiply), then the Python-double ratio
    elementwise in IEEE double (the same bits as float(a) / float(b))."""
    stakes_tao = S * config.total_subnet_stake
    stakes_units = (stakes_tao / 1000.0).numpy().astype(np.float64)  # float(x.item()): exact widening
    E_i = config.validator_emission_ratio * Dn
    emission = (E_i * config.total_epoch_emission).numpy().astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(stakes_units > 1e-6, emission / stakes_units, 0.0)


def _dividends_per_1000_tao(case: BaseCase, config: YumaConfig, S: torch.Tensor,
                            Dn: torch.Tensor) -> dict[str, list[float]]:
    """One run's dividend lists from [E, V] CPU tensors (O(E*V) output
    formatting, not the hot path)."""
    cols = _dividend_ratio(config, S, Dn).T.tolist()
    return {validator: cols[i] for i, validator in enumerate(case.validators)}


def _reward_key(config: YumaConfig) -> tuple:
    return (config.total_subnet_stake, config.validator_emission_ratio, config.total_epoch_emission)


def run_simulations(runs: list[SimulationRun], *, want_bonds: bool = True,
                    want_incentives: bool = True):
    """Run many simulations; runs that share (variant, E, V, M) go to the
    device as one batched engine call. Returns one (dividends, bonds, incentives)
    tuple per run, in order."""
    # the result lists are thousands of fresh containers (the sheet: 1512
    # dividend lists): the cyclic collector would sweep the process's whole
    # heap several times while they are built; they hold no cycles
    with _no_cyclic_gc():
        return _run_simulations(runs, want_bonds, want_incentives)


@contextmanager
def _no_cyclic_gc():
    enabled = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if enabled:
            gc.enable()


# stacked device inputs of small run groups, by the identity of their cases'
# packed inputs (built once per case and read only, cases.packed_inputs): the
# sheet restacks and uploads the same five groups on every call otherwise
_GROUP_INPUTS: dict = {}
_GROUP_INPUTS_MAX_ELEMS = 1 << 22  # W elements of a whole group; larger groups are stacked per call


def _group_inputs(packed: list, elems: int):
    """(W [E,N,V,M] and S [E,N,V] on the engine's device, S on the host);
    elems: the group's W elements."""
    src = tuple(t for p in packed for t in (p[2], p[3]))
    key = tuple(id(t) for t in src)
    if elems <= _GROUP_INPUTS_MAX_ELEMS:
        ent = _GROUP_INPUTS.get(key)
        if ent is not None and all(a is b for a, b in zip(ent[0], src)):
            return ent[1:]
    W = torch.stack([p[2] for p in packed], dim=1)
    S_host = torch.stack([p[3] for p in packed], dim=1).cpu()
    dev = engine.device()
    out = (W.to(device=dev, dtype=torch.float32).contiguous(),
           S_host.to(device=dev, dtype=torch.float32).contiguous(), S_host)
    if elems <= _GROUP_INPUTS_MAX_ELEMS:
        if len(_GROUP_INPUTS) >= 64:
            _GROUP_INPUTS.clear()
        _GROUP_INPUTS[key] = (src,) + out
    return out


_PLAIN = (int, type(None))


def _prefix_total(cs: np.ndarray, E: int, n: int):
    """sum(lst[:n]) of an E-entry list of floats from the running sums cs
    [E, V] of its values: Python's left-to-right double sum from int 0, i.e.
    the prefix's running sum (+0.0 turns a -0.0 into the +0.0 that 0 + -0.0
    gives) or the int 0 of an empty slice."""
    k = len(range(E)[:n])
    if k == 0:
        return [0] * cs.shape[1]
    return (cs[k - 1] + 0.0).tolist()


def _run_simulations(runs: list[SimulationRun], want_bonds: bool, want_incentives: bool,
                     totals: bool = False):
    """totals: each run's dividends as the sums of its first case.num_epochs
    per-epoch values, one per validator in case.validators order (the sheet's
    totals, the same bits as summing the lists) instead of the per-epoch
    lists, with no bonds or incentives."""
    groups: dict[tuple, list[int]] = defaultdict(list)
    packed = []
    for k, r in enumerate(runs):
        variant, reset_mode = resolve_version(r.yuma_version)
        W, S = r.case.packed_inputs()
        packed.append((variant, reset_mode, W, S))
        groups[(variant,) + tuple(W.shape)].append(k)

    results: list = [None] * len(runs)
    ckeys: dict[int, tuple] = {}  # per config object, for this call (the sheet shares 36 configs over 504 runs)
    # every group's engine run is queued before the first result is copied
    # back, so the device works through the later groups while the host
    # formats the earlier ones (the sheet: five groups)
    launched = []
    for (variant, E, V, M), idx in groups.items():
        params = []
        local: dict = {}  # (config object, reset fields) -> record, within the group
        for k in idx:
            r = runs[k]
            reset_mode = packed[k][1]
            cfg = r.yuma_config
            re_, ri_ = r.case.reset_bonds_epoch, r.case.reset_bonds_index
            plain = type(re_) in _PLAIN and type(ri_) in _PLAIN  # make_params_cached's memo rule
            lk = (id(cfg), reset_mode, re_, ri_) if plain else None
            rec = local.get(lk) if plain else None
            if rec is None:
                ck = ckeys.get(id(cfg))
                if ck is None:
                    ck = ckeys[id(cfg)] = engine.config_key(cfg)
                rec = engine.make_params_cached(variant, cfg, reset_mode=reset_mode, reset_epoch=re_,
                                                reset_index=ri_, n_miners=M, n_epochs=E, ckey=ck)
                if lk is not None:
                    local[lk] = rec
            params.append(rec)
        W, S, S_host = _group_inputs([packed[k] for k in idx], E * V * M * len(idx))
        launched.append((E, V, idx, S_host, engine.run(variant, params, W, S, want_hist=want_bonds)))
    for E, V, idx, S, res in launched:
        Dn = res.Dn.cpu()
        hist = res.B_hist.cpu() if want_bonds else None
        inc = res.I.cpu() if want_incentives else None
        # the dividend ratio of the whole group in one pass of the same
        # elementwise ops when its runs share the reward scalars (the sheet)
        ratio = None
        if len({_reward_key(runs[k].yuma_config) for k in idx}) == 1:
            ratio = _dividend_ratio(runs[idx[0]].yuma_config, S, Dn)  # [E, N, V]
        if totals:
            if ratio is not None:  # the group's prefix sums in one gather (the rows _prefix_total takes)
                csum = np.cumsum(ratio, axis=0)  # sequential, as sum()
                ks = [len(range(E)[:runs[k].case.num_epochs]) for k in idx]
                rows = (csum[[max(x - 1, 0) for x in ks], range(len(idx)), :] + 0.0).tolist()
            for j, k in enumerate(idx):
                r = runs[k]
                if ratio is not None:
                    tot = rows[j] if ks[j] > 0 else [0] * V
                else:
                    cs = np.cumsum(_dividend_ratio(r.yuma_config, packed[k][3].cpu(), Dn[:, j]), axis=0)
                    tot = _prefix_total(cs, E, r.case.num_epochs)
                results[k] = (tot, None, None)
            continue
        for j, k in enumerate(idx):
            r = runs[k]
            home = packed[k][2].device
            if ratio is not None:
                cols = ratio[:, j, :].T.tolist()
                div = {validator: cols[i] for i, validator in enumerate(r.case.validators)}
            else:
                div = _dividends_per_1000_tao(r.case, r.yuma_config, packed[k][3].cpu(), Dn[:, j])
            bonds = [hist[e, j].clone().to(home) for e in range(E)] if want_bonds else []
            incentives = [inc[e, j].clone().to(home) for e in range(E)] if want_incentives else []
            results[k] = (div, bonds, incentives)
    return results


def run_simulation(
    case: BaseCase,
    yuma_version: str,
    yuma_config: YumaConfig,
) -> tuple[dict[str, list[float]], list[torch.Tensor], list[torch.Tensor]]:
    """Runs the Yuma simulation for a given case and Yuma version, returning
    dividends, bonds and incentive data (reference simulation_utils.py:26-112)."""
    resolve_version(yuma_version)
    return run_simulations([SimulationRun(case, yuma_version, yuma_config)])[0]


SHEET_BOND_PENALTIES = (0, 0.5, 0.99, 1.0)  # scripts/total_dividends_sheet_generator.py:14


def sheet_yuma_versions() -> list[tuple[str, YumaParams]]:
    """The nine (version, YumaParams) pairs both reference scripts sweep
    (scripts/total_dividends_sheet_generator.py:25-48,
    scripts/charts_table_generator.py:27-47)."""
    from dataclasses import replace

    base = YumaParams()
    liquid = YumaParams(liquid_alpha=True)
    y4_liquid = replace(YumaParams(bond_alpha=0.025, alpha_high=0.99, alpha_low=0.9), liquid_alpha=True)
    n = _NAMES
    return [
        (n.YUMA_RUST, base), (n.YUMA, base), (n.YUMA_LIQUID, liquid), (n.YUMA2, base),
        (n.YUMA3, base), (n.YUMA31, base), (n.YUMA32, base), (n.YUMA4, base),
        (n.YUMA4_LIQUID, y4_liquid),
    ]


_STANDARDIZED = ["Validator A", "Validator B", "Validator C"]


def _sheet_runs(cases: list[BaseCase], yuma_versions, hyper: SimulationHyperparameters):
    for case in cases:
        if len(case.validators) != 3:
            raise ValueError(f"Case '{case.name}' does not have exactly 3 validators.")
    # one config per version, shared by every case's run (configs are read only)
    configs = [YumaConfig(simulation=hyper, yuma_params=params) for _, params in yuma_versions]
    return [
        SimulationRun(case, version, cfg)
        for case in cases
        for (version, _), cfg in zip(yuma_versions, configs)
    ]


def _sheet_frame(cases: list[BaseCase], yuma_versions, results) -> pd.DataFrame:
    """Rows of the dividend sheet from the runs' results (dividend lists), in
    _sheet_runs order (reference simulation_utils.py:341-381)."""
    results = iter(results)
    totals = []
    for case in cases:
        for _ in yuma_versions:
            dividends, _, _ = next(results)
            n = case.num_epochs
            totals.append([sum(dividends.get(v, [])[:n]) for v in case.validators])
    return _sheet_frame_totals(cases, yuma_versions, totals)


def _sheet_frame_totals(cases: list[BaseCase], yuma_versions, totals) -> pd.DataFrame:
    """The sheet from each run's total dividends (one per validator, in
    case.validators order): the totals of _calculate_total_dividends,
    reference charts_utils.py:15-45, with its zero-base warning (its
    percentage differences are not part of the sheet). With three distinct
    validators per case (validator i is standardised name i) and float totals
    the rows go into one float64 block: one frame construction instead of one
    column at a time (the same values, dtypes and CSV text); otherwise (the
    int 0 of an empty epoch range, no cases, repeated names) the frame is
    built from row dicts."""
    nv = len(yuma_versions)
    columns = ["Case"] + [f"{std} - {version}" for version, _ in yuma_versions for std in _STANDARDIZED]
    block = (bool(cases) and len(set(columns)) == len(columns)
             and all(len(set(c.validators)) == len(c.validators) == 3 for c in cases)
             and all(type(x) is float for t in totals for x in t))
    warn = "Warning: Base validator '{}' has zero or missing total dividends."
    it = iter(totals)
    if block:
        rows = []
        for case in cases:
            vs, bv = case.validators, case.base_validator
            bi = vs.index(bv) if bv in vs else None
            row: list = []
            for _ in range(nv):
                tot = next(it)
                if bi is None or tot[bi] == 0.0:
                    print(warn.format(bv))
                row += tot
            rows.append(row)
        df = pd.DataFrame(np.array(rows, dtype=np.float64), columns=columns[1:])
        df.insert(0, "Case", [case.name for case in cases])
        return df
    drows: list[dict[str, object]] = []
    for case in cases:
        std_of = dict(zip(case.validators, _STANDARDIZED))
        drow: dict[str, object] = {"Case": case.name}
        for version, _ in yuma_versions:
            tot = dict(zip(case.validators, next(it)))
            base = tot.get(case.base_validator)
            if base is None or base == 0.0:
                print(warn.format(case.base_validator))
            by_std = {std_of[v]: tot.get(v, 0.0) for v in case.validators}
            for std in _STANDARDIZED:
                drow[f"{std} - {version}"] = by_std.get(std, 0.0)
        drows.append(drow)
    df = pd.DataFrame(drows)
    return df[[c for c in columns if c in df.columns]]


def generate_total_dividends_table(
    cases: list[BaseCase],
    yuma_versions: list[tuple[str, YumaParams]],
    simulation_hyperparameters: SimulationHyperparameters,
) -> pd.DataFrame:
    """Total dividends per standardized validator and version (reference
    simulation_utils.py:319-381). All (case, version) runs are batched."""
    with _no_cyclic_gc():
        runs = _sheet_runs(cases, yuma_versions, simulation_hyperparameters)
        return _sheet_frame_totals(cases, yuma_versions, [d for d, _, _ in _run_simulations(runs, False, False, totals=True)])


def generate_total_dividends_tables(
    cases: list[BaseCase],
    yuma_versions: list[tuple[str, YumaParams]],
    simulation_hyperparameters: list[SimulationHyperparameters],
) -> list[pd.DataFrame]:
    """One dividend table per hyperparameter set (the sheet script's four
    bond penalties, scripts/total_dividends_sheet_generator.py:14-59), with the
    runs of ALL tables packed into one engine call per variant (config c5:
    504 runs in five launches sequences instead of twenty)."""
    with _no_cyclic_gc():
        per = [_sheet_runs(cases, yuma_versions, h) for h in simulation_hyperparameters]
        flat = [d for d, _, _ in _run_simulations([r for runs in per for r in runs], False, False, totals=True)]
        out, k = [], 0
        for runs in per:
            out.append(_sheet_frame_totals(cases, yuma_versions, flat[k:k + len(runs)]))
            k += len(runs)
    return out


from yuma_simulation._internal.html_tables import (  # noqa: E402,F401  (re-exported surface)
    _generate_draggable_html_table,
    _generate_ipynb_table,
)
