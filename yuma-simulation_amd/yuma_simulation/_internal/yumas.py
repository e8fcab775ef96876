"""Yuma epoch-step variants backed by the MI355X engine.

Drop-in for src/yuma_simulation/_internal/yumas.py: same config dataclasses
(with the same defaults and the same attribute flattening), same variant names,
same function signatures and the same result dictionaries (keys, dtypes,
Python-float vs tensor types). Every variant is one ``yuma_epoch`` C-ABI
call on the GPU (engine.run(single_call=True), every output requested);
nothing is computed on the CPU. Results come back on the device
of the input ``W`` (CPU in, CPU out — as the reference returns them).
"""

from __future__ import annotations

from dataclasses import dataclass, field, fields

import torch

from yuma_simulation._internal import engine


@dataclass
class SimulationHyperparameters:
    """Global knobs (reference yumas.py:7-14)."""

    kappa: float = 0.5
    bond_penalty: float = 1.0
    total_epoch_emission: float = 100.0
    validator_emission_ratio: float = 0.41
    total_subnet_stake: float = 1_000_000.0
    consensus_precision: int = 100_000


@dataclass
class YumaParams:
    """Per-variant knobs (reference yumas.py:17-26)."""

    bond_alpha: float = 0.1
    liquid_alpha: bool = False
    alpha_high: float = 0.9
    alpha_low: float = 0.7
    decay_rate: float = 0.1
    capacity_alpha: float = 0.1
    override_consensus_high: float | None = None
    override_consensus_low: float | None = None


@dataclass
class YumaConfig:
    """Both groups, with every field also readable as ``config.<name>``
    (reference yumas.py:29-45 copies them onto the instance)."""

    simulation: SimulationHyperparameters = field(default_factory=SimulationHyperparameters)
    yuma_params: YumaParams = field(default_factory=YumaParams)

    def __post_init__(self):
        # the reference copies asdict(group) onto the instance; every field is
        # an immutable scalar or None, so copying the attributes is the same
        for group in (self.simulation, self.yuma_params):
            for f in fields(group):
                setattr(self, f.name, getattr(group, f.name))


@dataclass(frozen=True)
class YumaSimulationNames:
    """Display names used as dispatch keys (reference yumas.py:48-58)."""

    YUMA_RUST: str = "Yuma 0 (subtensor)"
    YUMA: str = "Yuma 1 (paper)"
    YUMA_LIQUID: str = "Yuma 1 (paper) - liquid alpha on"
    YUMA2: str = "Yuma 2 (Adrian-Fish)"
    YUMA3: str = "Yuma 3 (Rhef)"
    YUMA31: str = "Yuma 3.1 (Rhef+reset)"
    YUMA32: str = "Yuma 3.2 (Rhef+conditional)"
    YUMA4: str = "Yuma 4 (Rhef+relative bonds)"
    YUMA4_LIQUID: str = "Yuma 4 (Rhef+relative bonds) - liquid alpha on"


# Keys of each variant's result, in the reference's order.
_COMMON = (
    "weight", "stake", "server_prerank", "server_consensus_weight",
    "consensus_clipped_weight", "server_rank", "server_incentive",
)
RESULT_KEYS = {
    engine.VARIANT_RUST: _COMMON + (
        "server_trust", "validator_trust", "validator_bond", "validator_ema_bond",
        "validator_reward", "validator_reward_normalized", "bond_alpha", "alpha_a", "alpha_b"),
    engine.VARIANT_YUMA1: _COMMON + (
        "server_trust", "validator_trust", "weight_for_bond", "validator_bond",
        "validator_ema_bond", "validator_reward", "validator_reward_normalized",
        "bond_alpha", "alpha_a", "alpha_b"),
    engine.VARIANT_YUMA3: _COMMON + (
        "server_trust", "validator_trust", "validator_bonds", "validator_reward",
        "validator_reward_normalized"),
    engine.VARIANT_YUMA4: _COMMON + (
        "validator_bonds", "validator_reward", "validator_reward_normalized"),
}
RESULT_KEYS[engine.VARIANT_YUMA2] = RESULT_KEYS[engine.VARIANT_YUMA1]


def _epoch(variant: int, W: torch.Tensor, S: torch.Tensor, B_old, config: YumaConfig,
           W_prev=None, maxint: int = 2**64 - 1) -> dict:
    if W.dim() != 2:
        raise ValueError(f"W must be [validators, miners], got shape {tuple(W.shape)}")
    V, M = W.shape
    if S.dim() != 1 or S.shape[0] != V:
        raise ValueError(f"S must be [{V}], got shape {tuple(S.shape)}")
    if B_old is not None and tuple(B_old.shape) != (V, M):
        raise ValueError(f"B_old must be [{V}, {M}], got {tuple(B_old.shape)}")
    if W_prev is not None and tuple(W_prev.shape) != (V, M):
        raise ValueError(f"W_prev must be [{V}, {M}], got {tuple(W_prev.shape)}")
    home = W.device
    prm = engine.make_params(variant, config, maxint=maxint)
    liquid = prm.liquid_mode != engine.LIQUID_OFF
    want = ["R", "P", "T", "Tv", "Sn", "Wn", "Wc", "D"]
    if variant in (engine.VARIANT_YUMA1, engine.VARIANT_YUMA2):
        want += ["Wb", "B_inst"]
    if variant == engine.VARIANT_RUST:
        want += ["B_inst"]
    if liquid:
        want += ["bond_alpha", "alpha_ab"]
    res = engine.run(
        variant, [prm], W.reshape(1, 1, V, M), S.reshape(1, 1, V),
        None if B_old is None else B_old.reshape(1, V, M),
        None if W_prev is None else W_prev.reshape(1, V, M),
        want=tuple(want), single_call=True,
    )
    x = res.extra

    def back(t: torch.Tensor, *shape) -> torch.Tensor:
        return t.reshape(*shape).to(home)

    d = {
        "weight": back(x["Wn"], V, M),
        "stake": back(x["Sn"], V),
        "server_prerank": back(x["P"], M),
        "server_consensus_weight": back(res.C, M),
        "consensus_clipped_weight": back(x["Wc"], V, M),
        "server_rank": back(x["R"], M),
        "server_incentive": back(res.I, M),
        "server_trust": back(x["T"], M),
        "validator_trust": back(x["Tv"], V),
        "validator_reward": back(x["D"], V),
        "validator_reward_normalized": back(res.Dn, V),
    }
    bond_state = back(res.B_final, V, M)
    if variant in (engine.VARIANT_YUMA3, engine.VARIANT_YUMA4):
        d["validator_bonds"] = bond_state
    else:
        if variant != engine.VARIANT_RUST:
            d["weight_for_bond"] = back(x["Wb"], V, M)
        d["validator_bond"] = back(x["B_inst"], V, M)
        if variant != engine.VARIANT_RUST and B_old is None:
            d["validator_ema_bond"] = d["validator_bond"]  # aliased (yumas.py:258)
        else:
            d["validator_ema_bond"] = bond_state
        if liquid:
            d["bond_alpha"] = back(x["bond_alpha"], M)
            if prm.liquid_mode == engine.LIQUID_CONST_AB:
                a, b = _const_ab(config)
                d["alpha_a"], d["alpha_b"] = a, b
            else:
                ab = x["alpha_ab"].reshape(2).to(home)
                d["alpha_a"], d["alpha_b"] = ab[0].clone(), ab[1].clone()
        else:
            d["bond_alpha"] = config.bond_alpha
            d["alpha_a"] = d["alpha_b"] = torch.tensor(float("nan"))
    return {k: d[k] for k in RESULT_KEYS[variant]}


def _const_ab(config) -> tuple[float, float]:
    import math

    ln_high = math.log(1 / config.alpha_high - 1)
    ln_low = math.log(1 / config.alpha_low - 1)
    a = (ln_high - ln_low) / (config.override_consensus_low - config.override_consensus_high)
    return a, ln_low + a * config.override_consensus_low


def YumaRust(W: torch.Tensor, S: torch.Tensor, B_old: torch.Tensor | None = None,
             config: YumaConfig = YumaConfig()) -> dict[str, torch.Tensor | str | float]:
    """Subtensor's Yuma (reference yumas.py:61-172): fp64 consensus, column-
    normalised bonds and EMA bonds."""
    return _epoch(engine.VARIANT_RUST, W, S, B_old, config)


def Yuma(W: torch.Tensor, S: torch.Tensor, B_old: torch.Tensor | None = None,
         config: YumaConfig = YumaConfig()) -> dict[str, torch.Tensor | None | float]:
    """Yuma 1 / paper (reference yumas.py:175-282): bond-penalised weights,
    column-normalised bonds, EMA (fixed or liquid alpha)."""
    return _epoch(engine.VARIANT_YUMA1, W, S, B_old, config)


def Yuma2(W: torch.Tensor, W_prev: torch.Tensor | None, S: torch.Tensor,
          B_old: torch.Tensor | None = None,
          config: YumaConfig = YumaConfig()) -> dict[str, torch.Tensor | None | float]:
    """Yuma 2 / Adrian-Fish (reference yumas.py:285-396): clips and bonds the
    previous epoch's normalised weights ``W_prev`` (``W`` itself when None)."""
    return _epoch(engine.VARIANT_YUMA2, W, S, B_old, config, W_prev=W_prev)


def Yuma3(W: torch.Tensor, S: torch.Tensor, B_old: torch.Tensor | None = None,
          config: YumaConfig = YumaConfig(),
          maxint: int = 2**64 - 1) -> dict[str, torch.Tensor | None | float]:
    """Yuma 3 / Rhef (reference yumas.py:399-491): capacity-purchase bonds.
    Like the reference it ignores bond_alpha, liquid_alpha and bond_penalty."""
    return _epoch(engine.VARIANT_YUMA3, W, S, B_old, config, maxint=maxint)


def Yuma4(W: torch.Tensor, S: torch.Tensor, B_old: torch.Tensor | None = None,
          config: YumaConfig = YumaConfig()) -> dict[str, torch.Tensor | None | float]:
    """Yuma 4 / Rhef + relative bonds (reference yumas.py:494-606)."""
    return _epoch(engine.VARIANT_YUMA4, W, S, B_old, config)
