"""torch-CPU restatement of the Yuma epoch step (all five variants) and of
run_simulation's epoch loop -- TEST AND BASELINE INFRASTRUCTURE, not product
code.

Only tests/ and bench.py's cpu_baseline leg import this module (SURVEY §8d:
"time the build's CPU restatement ... (i) reference-structured, (ii)
vectorised torch-CPU"). It restates src/yuma_simulation/_internal/yumas.py
with the same torch CPU operations in the same order, so it rounds exactly as
the reference does: tests/test_oracle_golden.py checks it BIT-FOR-BIT against
the goldens captured from the reference (tests/golden/).

Two consensus forms (yumas.py:195-209 / :420-434 / :514-528):
  structured  one Python bisection loop per miner column over a 1-D column
              view, as the reference runs it (single-threaded Python, ~93 % of
              the reference's epoch time);
  vectorised  the same bisection for all columns at once: each iteration is
              one [V, M] compare + column sum (torch intra-op threads).
The two give the same C whenever the stake sums are order-independent (the
benchmark's dyadic stakes); on generic floats the vectorised column sums run
in another order (the tie window, oracle.yuma_oracle.tie_columns).
"""

from __future__ import annotations

import math

import torch

F32 = torch.float32


def _iterations(precision) -> int:
    thr = 1 / precision
    hi, lo, n = 1.0, 0.0, 0
    while (hi - lo) > thr:
        hi = (hi + lo) / 2.0
        n += 1
    return n


def consensus_structured(W: torch.Tensor, S: torch.Tensor, kappa: float, precision) -> torch.Tensor:
    """Per-column bisection with Python-double bounds (yumas.py:420-434)."""
    thr = 1 / precision
    out = torch.zeros(W.shape[1])
    for m, column in enumerate(W.T):
        lo, hi = 0.0, 1.0
        while (hi - lo) > thr:
            mid = (hi + lo) / 2.0
            stake_above = (column > mid) * S
            if stake_above.sum() > kappa:
                lo = mid
            else:
                hi = mid
        out[m] = hi
    return out


def consensus_vectorised(W: torch.Tensor, S: torch.Tensor, kappa: float, precision) -> torch.Tensor:
    """All columns' bisections in lock-step: fp64 bounds (the Python doubles),
    fp32 midpoint compare and stake sum, fp32 kappa -- the reference's
    per-column decisions, evaluated for every column per iteration."""
    M = W.shape[1]
    lo = torch.zeros(M, dtype=torch.float64)
    hi = torch.ones(M, dtype=torch.float64)
    k32 = torch.tensor(kappa, dtype=F32)
    Sc = S.view(-1, 1)
    for _ in range(_iterations(precision)):
        mid = (hi + lo) / 2.0
        above = W > mid.to(F32).view(1, -1)
        up = (above * Sc).sum(dim=0) > k32
        lo = torch.where(up, mid, lo)
        hi = torch.where(up, hi, mid)
    return hi.to(F32)


def _liquid_bond_alpha(C: torch.Tensor, cfg):
    """The liquid-alpha block every variant but Yuma3 carries (yumas.py:118-140,
    :231-253, :345-367, :546-568). Returns (bond_alpha, a, b)."""
    high = cfg.override_consensus_high if cfg.override_consensus_high is not None else C.quantile(0.75)
    low = cfg.override_consensus_low if cfg.override_consensus_low is not None else C.quantile(0.25)
    if high == low:
        high = C.quantile(0.99)
    ln_hi = math.log(1 / cfg.alpha_high - 1)
    ln_lo = math.log(1 / cfg.alpha_low - 1)
    a = (ln_hi - ln_lo) / (low - high)
    b = ln_lo + a * low
    alpha = 1 / (1 + math.e ** (-a * C + b))
    return 1 - torch.clamp(alpha, cfg.alpha_low, cfg.alpha_high), a, b


VARIANTS = ("rust", "yuma1", "yuma2", "yuma3", "yuma4")


def epoch(variant: str, W: torch.Tensor, S: torch.Tensor, B_old: torch.Tensor | None, cfg,
          consensus: str = "structured", maxint: int = 2**64 - 1, W_prev: torch.Tensor | None = None) -> dict:
    """One YumaRust (yumas.py:61-172), Yuma (:175-282), Yuma2 (:285-396),
    Yuma3 (:399-491) or Yuma4 (:494-606) call on CPU tensors, returning the
    reference's result dict (same keys, dtypes and Python-float entries)."""
    if variant not in VARIANTS:
        raise ValueError(f"torch_cpu restates {VARIANTS}, not {variant}")
    Wn = (W.T / (W.sum(dim=1) + 1e-6)).T
    if variant == "yuma2" and W_prev is None:
        W_prev = Wn
    Sn = S / S.sum()
    P = (Sn.view(-1, 1) * Wn).sum(dim=0)
    find = consensus_structured if consensus == "structured" else consensus_vectorised
    C = find(Wn, Sn, cfg.kappa, cfg.consensus_precision)
    if variant == "rust":  # C is an fp64 tensor there (yumas.py:81); the bisection points are exact
        C = C.to(torch.float64)
    C = (C / C.sum() * 65_535).int() / 65_535
    Wc = torch.min(W_prev if variant == "yuma2" else Wn, C)
    R = (Sn.view(-1, 1) * Wc).sum(dim=0)
    I = (R / R.sum()).nan_to_num(0)
    T = (R / P).nan_to_num(0)
    Tv = Wc.sum(dim=1) / Wn.sum(dim=1)
    out = {"weight": Wn, "stake": Sn, "server_prerank": P, "server_consensus_weight": C,
           "consensus_clipped_weight": Wc, "server_rank": R, "server_incentive": I}
    if variant in ("rust", "yuma1", "yuma2"):
        if variant == "rust":
            B = Sn.view(-1, 1) * Wc
            B = B / (B.sum(dim=0) + 1e-6)
            B = torch.nan_to_num(B)
        else:
            Wb = (1 - cfg.bond_penalty) * (W_prev if variant == "yuma2" else Wn) + cfg.bond_penalty * Wc
            B = Sn.view(-1, 1) * Wb / (Sn.view(-1, 1) * Wb).sum(dim=0)
            B = B.nan_to_num(0)
        a = b = torch.tensor(float("nan"))
        ba = cfg.bond_alpha
        if cfg.liquid_alpha:
            ba, a, b = _liquid_bond_alpha(C, cfg)
        if B_old is not None:
            Bema = ba * B + (1 - ba) * B_old
        else:
            Bema = B.clone() if variant == "rust" else B
        if variant == "rust":
            Bema = Bema / (Bema.sum(dim=0) + 1e-6)
            Bema = torch.nan_to_num(Bema)
        D = (Bema * I).sum(dim=1)
        out.update(server_trust=T, validator_trust=Tv)
        if variant != "rust":
            out["weight_for_bond"] = Wb
        out.update(validator_bond=B, validator_ema_bond=Bema)
        out["validator_reward"] = D
        out["validator_reward_normalized"] = D / (D.sum() + 1e-6)
        out.update(bond_alpha=ba, alpha_a=a, alpha_b=b)
        return out
    Bo = torch.zeros_like(Wn) if B_old is None else B_old
    if variant == "yuma3":
        cap = Sn.unsqueeze(1) * maxint
        room = torch.clamp(cap - Bo, min=0.0)
        buy = torch.min((cfg.capacity_alpha * (Sn * maxint)).unsqueeze(1), room)
        B = torch.min((1 - cfg.decay_rate) * Bo + buy * Wn, cap)
        D = (B * I).sum(dim=1)
        out.update(server_trust=T, validator_trust=Tv, validator_bonds=B)
    else:
        ba = cfg.bond_alpha
        if cfg.liquid_alpha:
            ba, _, _ = _liquid_bond_alpha(C, cfg)
        Bd = Bo * (1 - ba)
        room = torch.clamp(1.0 - Bd, min=0.0)
        B = torch.clamp(Bd + torch.min(ba * Wn, room), max=1.0)
        D = Sn * (B * I).sum(dim=1)
        out.update(validator_bonds=B)
    out["validator_reward"] = D
    out["validator_reward_normalized"] = D / (D.sum() + 1e-6)
    return out


def state_key(variant: str) -> str:
    return "validator_bonds" if variant in ("yuma3", "yuma4") else "validator_ema_bond"


def run(variant: str, W_epochs: torch.Tensor, S_epochs: torch.Tensor, cfg, consensus: str = "structured",
        epochs: int | None = None) -> dict:
    """The run_simulation loop (simulation_utils.py:52-110) without resets,
    for the benchmark versions ("Yuma 3 (Rhef)", "Yuma 4 ..." with resets off)."""
    B = None
    Dn, C = [], []
    for t in range(W_epochs.shape[0] if epochs is None else epochs):
        r = epoch(variant, W_epochs[t], S_epochs[t], B, cfg, consensus)
        B = r["validator_bonds"]
        Dn.append(r["validator_reward_normalized"])
        C.append(r["server_consensus_weight"])
    return {"Dn": torch.stack(Dn), "C": torch.stack(C), "B": B}


# version string -> (variant, reset rule) of run_simulation's dispatch (simulation_utils.py:52-93)
VERSIONS = {
    "Yuma 0 (subtensor)": ("rust", None),
    "Yuma 1 (paper)": ("yuma1", None),
    "Yuma 1 (paper) - liquid alpha on": ("yuma1", None),
    "Yuma 2 (Adrian-Fish)": ("yuma2", None),
    "Yuma 3 (Rhef)": ("yuma3", None),
    "Yuma 3.1 (Rhef+reset)": ("yuma3", "always"),
    "Yuma 3.2 (Rhef+conditional)": ("yuma3", "if_zero"),
    "Yuma 4 (Rhef+relative bonds)": ("yuma4", "if_zero"),
    "Yuma 4 (Rhef+relative bonds) - liquid alpha on": ("yuma4", "if_zero"),
}


def run_simulation(version: str, weights_epochs, stakes_epochs, cfg, num_epochs: int, validators,
                   reset_bonds_epoch=None, reset_bonds_index=None, consensus: str = "structured"):
    """run_simulation (simulation_utils.py:26-112) on CPU torch: the epoch
    loop with the bond resets and the fp64 dividend-per-1000-tao lists.
    Returns (dividends_per_validator, bonds_per_epoch, incentives_per_epoch)."""
    if version not in VERSIONS:
        raise ValueError("Invalid Yuma function.")
    variant, reset = VERSIONS[version]
    div = {v: [] for v in validators}
    bonds, incentives = [], []
    B_state = W_prev = scw = None
    for epoch_i in range(num_epochs):
        W, S = weights_epochs[epoch_i], stakes_epochs[epoch_i]
        units = S * cfg.total_subnet_stake / 1000.0
        if reset is not None and B_state is not None and epoch_i == reset_bonds_epoch:
            if reset == "always" or (scw is not None and scw[reset_bonds_index] == 0.0):
                B_state[:, reset_bonds_index] = 0.0
        r = epoch(variant, W, S, B_state, cfg, consensus, W_prev=W_prev)
        B_state = r[state_key(variant)]
        if variant == "yuma2":
            W_prev = r["weight"]
        scw = r["server_consensus_weight"]
        emis = cfg.validator_emission_ratio * r["validator_reward_normalized"] * cfg.total_epoch_emission
        for i, v in enumerate(validators):
            su = float(units[i].item())
            ei = float(emis[i].item())
            div[v].append(ei / su if su > 1e-6 else 0.0)
        bonds.append(B_state.clone())
        incentives.append(r["server_incentive"])
    return div, bonds, incentives
