"""CPU oracle for the Yuma epoch step — TEST INFRASTRUCTURE, not product code.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline. The
product path (yuma_simulation on libyuma_hip.so) never calls it.

What it is: a vectorised numpy restatement of the reference algorithm,
op by op in fp32, written from the reference source
(src/yuma_simulation/_internal/yumas.py, simulation_utils.py). Each function
cites the lines it restates. It is pinned against golden fixtures captured
from the reference itself (tests/golden/make_golden.py, run in the build
container where /root/reference is importable): see tests/test_oracle_golden.py.

Rounding model (torch CPU semantics the reference runs under, probed):
  * a Python float meeting an fp32 tensor is rounded to fp32 first;
  * `py / t` is `reciprocal(t) * py`;
  * `math.e ** t` is `pow(fp32(e), t)`;
  * torch.quantile: rank = q * (n - 1) in fp32, lerp in FMA form;
  * torch.min / clamp propagate NaN; nan_to_num maps +-inf to +-FLT_MAX.
Summation order differs from torch (numpy pairwise); that is within the
stated tolerance and exact on the exactness-friendly synthetic inputs.
"""

from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

F32 = np.float32
FLT_MAX = np.finfo(np.float32).max
E32 = F32(math.e)

RUST, YUMA1, YUMA2, YUMA3, YUMA4 = "rust", "yuma1", "yuma2", "yuma3", "yuma4"

VERSIONS = {
    # simulation_utils.py:52-93 dispatch: version -> (variant, reset rule)
    "Yuma 0 (subtensor)": (RUST, None),
    "Yuma 1 (paper)": (YUMA1, None),
    "Yuma 1 (paper) - liquid alpha on": (YUMA1, None),
    "Yuma 2 (Adrian-Fish)": (YUMA2, None),
    "Yuma 3 (Rhef)": (YUMA3, None),
    "Yuma 3.1 (Rhef+reset)": (YUMA3, "always"),
    "Yuma 3.2 (Rhef+conditional)": (YUMA3, "if_zero_c"),
    "Yuma 4 (Rhef+relative bonds)": (YUMA4, "if_zero_c"),
    "Yuma 4 (Rhef+relative bonds) - liquid alpha on": (YUMA4, "if_zero_c"),
}


# ---------------------------------------------------------------------------
# scalar helpers
# ---------------------------------------------------------------------------
def _round_f32(x: Fraction) -> np.float32:
    """Correctly rounded (nearest-even) fp32 of an exact rational."""
    if x == 0:
        return F32(0.0)
    sign = -1 if x < 0 else 1
    x = abs(x)
    e = x.numerator.bit_length() - x.denominator.bit_length()
    if Fraction(2) ** e > x:
        e -= 1
    elif Fraction(2) ** (e + 1) <= x:
        e += 1
    e = max(e, -126)
    scaled = x * Fraction(2) ** (23 - e)
    n = scaled.numerator // scaled.denominator
    rem = scaled - n
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and n % 2 == 1):
        n += 1
    val = float(n) * 2.0 ** (e - 23)
    return F32(sign * val)


def fma32(a, b, c) -> np.float32:
    """fp32 fused multiply-add with a single rounding."""
    a, b, c = F32(a), F32(b), F32(c)
    if not (np.isfinite(a) and np.isfinite(b) and np.isfinite(c)):
        return F32(np.float64(a) * np.float64(b) + np.float64(c))
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def tmin(a, b):
    """torch.minimum semantics (NaN propagates)."""
    a, b = np.broadcast_arrays(np.asarray(a, F32), np.asarray(b, F32))
    out = np.minimum(a, b)  # np.minimum propagates NaN as torch does
    return out.astype(F32)


def tmax(a, b):
    a, b = np.broadcast_arrays(np.asarray(a, F32), np.asarray(b, F32))
    return np.maximum(a, b).astype(F32)


def nan_to_num(x, nan=0.0):
    return np.nan_to_num(np.asarray(x, F32), nan=F32(nan), posinf=FLT_MAX, neginf=-FLT_MAX).astype(F32)


def quantile(C: np.ndarray, q: float) -> np.float32:
    """torch.quantile(C, q), linear interpolation (ATen Sorting.cpp +
    the FMA lerp of the vectorised kernel), for a NaN-free 1-D fp32 tensor."""
    s = np.sort(C.astype(F32))
    n = s.shape[0]
    rank = F32(F32(q) * F32(n - 1))
    lo = int(rank)
    hi = int(math.ceil(float(rank)))
    w = F32(rank - F32(lo))
    a, b = s[lo], s[hi]
    diff = F32(b - a)
    if abs(float(w)) < 0.5:
        return fma32(w, diff, a)
    return fma32(-diff, F32(F32(1.0) - w), b)


def bisect_iterations(precision) -> int:
    thr = 1 / precision
    hi, lo, n = 1.0, 0.0, 0
    while (hi - lo) > thr:
        hi = (hi + lo) / 2.0
        n += 1
    return n


# ---------------------------------------------------------------------------
# the epoch step
# ---------------------------------------------------------------------------
def consensus(Wn: np.ndarray, S: np.ndarray, kappa: float, precision, as_double: bool):
    """Per-column stake-weighted kappa bisection (yumas.py:195-209; YumaRust
    :81-95 keeps C in fp64), vectorised over the miner columns."""
    V, M = Wn.shape
    lo = np.zeros(M, dtype=np.float64)
    hi = np.ones(M, dtype=np.float64)
    k32 = F32(kappa)
    Sc = S.astype(F32)[:, None]
    zero = F32(0.0)
    for _ in range(bisect_iterations(precision)):
        mid = (hi + lo) / 2.0
        midf = mid.astype(F32)
        sums = np.where(Wn > midf[None, :], Sc, zero).sum(axis=0, dtype=F32)
        up = sums > k32
        lo = np.where(up, mid, lo)
        hi = np.where(up, hi, mid)
    return hi if as_double else hi.astype(F32)


def tie_columns(W, S, kappa: float, precision, as_double: bool = False, ulps: int = 64) -> np.ndarray:
    """Miner columns whose consensus level depends on summation ORDER, so
    that two correct fp32 implementations (torch's CPU kernels, this numpy
    port, the HIP engine) may legitimately disagree on them.

    The reference decides `(W > mid) @ S > kappa` (yumas.py:203-204), sums
    W's rows (:186) and C (:211) in fp32, in torch's order. A column is
    flagged when, on the bisection path this oracle takes, either
      * the exact stake sum lies within V * 2^-24 of fp32(kappa) (the bound
        on any fp32 summation order of <= V terms in [0, 1]), or
      * a validator with stake has a normalised weight within `ulps` ulps of
        the midpoint (the row sums, hence W / rowsum, differ by order);
    or the quantisation `C / sum(C) * 65535` lies within `ulps` ulps of an
    integer (sum(C) differs by order). Outside these columns C must be
    bit-equal. Returns a bool mask [M]."""
    W = np.asarray(W, F32)
    S = np.asarray(S, F32)
    V, M = W.shape
    rs = W.sum(axis=1, dtype=F32)
    Wn = (W / (rs + F32(1e-6))[:, None]).astype(F32)
    Sn = (S / S.sum(dtype=F32)).astype(F32)
    staked = Sn > 0
    k32 = np.float64(F32(kappa))
    win = V * 2.0 ** -24
    Sc = Sn[:, None]
    S64 = Sn.astype(np.float64)
    lo = np.zeros(M, dtype=np.float64)
    hi = np.ones(M, dtype=np.float64)
    flag = np.zeros(M, dtype=bool)
    for _ in range(bisect_iterations(precision)):
        mid = (hi + lo) / 2.0
        midf = mid.astype(F32)
        above = Wn > midf[None, :]
        exact = (np.where(above, S64[:, None], 0.0)).sum(axis=0)
        flag |= np.abs(exact - k32) <= win
        near = np.abs(Wn.astype(np.float64) - midf[None, :]) <= ulps * np.spacing(midf)[None, :]
        flag |= (near & staked[:, None]).any(axis=0)
        sums = np.where(above, Sc, F32(0.0)).sum(axis=0, dtype=F32)
        up = sums > F32(kappa)
        lo = np.where(up, mid, lo)
        hi = np.where(up, hi, mid)
    c = hi if as_double else hi.astype(F32)
    x = (c.astype(np.float64) / c.astype(np.float64).sum()) * 65535.0
    frac_dist = np.abs(x - np.round(x))
    flag |= (frac_dist <= ulps * np.spacing(x.astype(F32)).astype(np.float64)) & (x > 0)
    return flag


def quantise(C_raw: np.ndarray, as_double: bool) -> np.ndarray:
    """(C / C.sum() * 65535).int() / 65535 (yumas.py:211; :97 in fp64)."""
    if as_double:
        q = (C_raw / C_raw.sum() * 65535.0).astype(np.int32)
    else:
        c = C_raw.astype(F32)
        q = (c / c.sum(dtype=F32) * F32(65535.0)).astype(F32).astype(np.int32)
    return (q.astype(F32) / F32(65535.0)).astype(F32)


def liquid_alpha(C: np.ndarray, cfg):
    """yumas.py:231-253 (and copies :118-140, :345-367, :546-568). Returns
    (bond_alpha [M] fp32, a, b) where a/b are fp32 scalars, or Python floats
    when both consensus overrides are given and differ (pure-Python path)."""
    ch_o = cfg.override_consensus_high
    cl_o = cfg.override_consensus_low
    ch = ch_o if ch_o is not None else quantile(C, 0.75)
    cl = cl_o if cl_o is not None else quantile(C, 0.25)
    both_py = ch_o is not None and cl_o is not None
    if both_py:
        eq = ch == cl
    else:
        eq = F32(ch) == F32(cl)
    if eq:
        ch = quantile(C, 0.99)
        both_py = False
    ln_high = math.log(1 / cfg.alpha_high - 1)
    ln_low = math.log(1 / cfg.alpha_low - 1)
    if both_py:
        a = (ln_high - ln_low) / (cl - ch)
        b = ln_low + a * cl
        a32, b32 = F32(a), F32(b)
        a_out, b_out = a, b
    else:
        d = F32(F32(cl) - F32(ch))
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            a32 = F32(F32(F32(1.0) / d) * F32(ln_high - ln_low))
            b32 = F32(F32(ln_low) + F32(a32 * F32(cl)))
        a_out, b_out = a32, b32
    with np.errstate(over="ignore", invalid="ignore"):
        x = (F32(-a32) * C).astype(F32)
        y = (x + b32).astype(F32)
        p = np.power(E32, y).astype(F32)
        alpha = (F32(1.0) / (F32(1.0) + p).astype(F32)).astype(F32)
    clamped = tmin(tmax(alpha, F32(cfg.alpha_low)), F32(cfg.alpha_high))
    return (F32(1.0) - clamped).astype(F32), a_out, b_out


def epoch(variant: str, W, S, B_old=None, cfg=None, W_prev=None, maxint: int = 2**64 - 1) -> dict:
    """One epoch of a Yuma variant; returns the reference's result dict with
    numpy values. variant in {rust, yuma1, yuma2, yuma3, yuma4}."""
    W = np.asarray(W, F32)
    S = np.asarray(S, F32)
    V, M = W.shape
    # === Weight / Stake / Prerank === (yumas.py:186-192 and copies)
    rs = W.sum(axis=1, dtype=F32)
    Wn = (W / (rs + F32(1e-6))[:, None]).astype(F32)
    Sn = (S / S.sum(dtype=F32)).astype(F32)
    P = (Sn[:, None] * Wn).astype(F32).sum(axis=0, dtype=F32)
    # === Consensus ===
    as_double = variant == RUST
    C = quantise(consensus(Wn, Sn, cfg.kappa, cfg.consensus_precision, as_double), as_double)
    # === Clip / Rank / Incentive / Trust === (yumas.py:214-224; Yuma2 :328)
    if variant == YUMA2:
        Wsrc = Wn if W_prev is None else np.asarray(W_prev, F32)
    else:
        Wsrc = Wn
    Wc = tmin(Wsrc, C[None, :])
    R = (Sn[:, None] * Wc).astype(F32).sum(axis=0, dtype=F32)
    with np.errstate(divide="ignore", invalid="ignore"):
        I = nan_to_num(R / R.sum(dtype=F32), 0.0)
        T = nan_to_num(R / P, 0.0)
        Tv = (Wc.sum(axis=1, dtype=F32) / Wn.sum(axis=1, dtype=F32)).astype(F32)
    out = {
        "weight": Wn, "stake": Sn, "server_prerank": P, "server_consensus_weight": C,
        "consensus_clipped_weight": Wc, "server_rank": R, "server_incentive": I,
    }
    liquid = bool(cfg.liquid_alpha) and variant != YUMA3
    if liquid:
        ba, a, b = liquid_alpha(C, cfg)
        ba_row = ba[None, :]
        omba = (F32(1.0) - ba_row).astype(F32)
    else:
        ba, a, b = cfg.bond_alpha, float("nan"), float("nan")
        ba_row = F32(cfg.bond_alpha)
        omba = F32(1 - cfg.bond_alpha)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        if variant == RUST:  # yumas.py:113-153
            B = (Sn[:, None] * Wc).astype(F32)
            B = nan_to_num(B / (B.sum(axis=0, dtype=F32) + F32(1e-6)))
            if B_old is not None:
                Bema = ((ba_row * B).astype(F32) + (omba * np.asarray(B_old, F32)).astype(F32)).astype(F32)
            else:
                Bema = B.copy()
            Bema = nan_to_num(Bema / (Bema.sum(axis=0, dtype=F32) + F32(1e-6)))
            D = (Bema * I).astype(F32).sum(axis=1, dtype=F32)
            out.update(server_trust=T, validator_trust=Tv, validator_bond=B, validator_ema_bond=Bema)
        elif variant in (YUMA1, YUMA2):  # yumas.py:227-262 / :341-376
            Wb = ((F32(1 - cfg.bond_penalty) * Wsrc).astype(F32)
                  + (F32(cfg.bond_penalty) * Wc).astype(F32)).astype(F32)
            num = (Sn[:, None] * Wb).astype(F32)
            B = nan_to_num(num / num.sum(axis=0, dtype=F32), 0.0)
            if B_old is not None:
                Bema = ((ba_row * B).astype(F32) + (omba * np.asarray(B_old, F32)).astype(F32)).astype(F32)
            else:
                Bema = B
            D = (Bema * I).astype(F32).sum(axis=1, dtype=F32)
            out.update(server_trust=T, validator_trust=Tv, weight_for_bond=Wb, validator_bond=B,
                       validator_ema_bond=Bema)
        elif variant == YUMA3:  # yumas.py:452-476
            Bo = np.zeros_like(Wn) if B_old is None else np.asarray(B_old, F32)
            cap = (Sn * F32(float(maxint))).astype(F32)[:, None]
            rem = tmax((cap - Bo).astype(F32), F32(0.0))
            pc = tmin((F32(cfg.capacity_alpha) * cap).astype(F32), rem)
            purchase = (pc * Wn).astype(F32)
            B = ((F32(1 - cfg.decay_rate) * Bo).astype(F32) + purchase).astype(F32)
            B = tmin(B, cap)
            D = (B * I).astype(F32).sum(axis=1, dtype=F32)
            out.update(server_trust=T, validator_trust=Tv, validator_bonds=B)
        else:  # YUMA4, yumas.py:570-593
            Bo = np.zeros_like(Wn) if B_old is None else np.asarray(B_old, F32)
            Bd = (Bo * omba).astype(F32)
            rem = tmax((F32(1.0) - Bd).astype(F32), F32(0.0))
            pi = (ba_row * Wn).astype(F32)
            B = tmin((Bd + tmin(pi, rem)).astype(F32), F32(1.0))
            D = (Sn * (B * I).astype(F32).sum(axis=1, dtype=F32)).astype(F32)
            out.update(validator_bonds=B)
        Dn = (D / (D.sum(dtype=F32) + F32(1e-6))).astype(F32)
    out["validator_reward"] = D
    out["validator_reward_normalized"] = Dn
    if variant in (RUST, YUMA1, YUMA2):
        out.update(bond_alpha=ba, alpha_a=a, alpha_b=b)
    return out


def state_key(variant: str) -> str:
    return "validator_bonds" if variant in (YUMA3, YUMA4) else "validator_ema_bond"


def run(version: str, W_epochs, S_epochs, cfg, reset_epoch=None, reset_index=None,
        validators=None):
    """The epoch loop of run_simulation (simulation_utils.py:26-112).
    Returns dict with per-epoch arrays Dn [E,V], C [E,M], I [E,M], B [E,V,M]
    and, if `validators` is given, the dividends-per-1000-tao lists."""
    if version not in VERSIONS:
        raise ValueError("Invalid Yuma function.")
    variant, reset = VERSIONS[version]
    W_epochs = np.asarray(W_epochs, F32)
    S_epochs = np.asarray(S_epochs, F32)
    E = W_epochs.shape[0]
    B_state = None
    W_prev = None
    C_prev = None
    Dn, Cs, Is, Bs = [], [], [], []
    for epoch_i in range(E):
        if B_state is not None and epoch_i == reset_epoch and reset is not None:
            fire = reset == "always" or (C_prev is not None and C_prev[reset_index] == 0.0)
            if fire:
                B_state = B_state.copy()
                B_state[:, reset_index] = 0.0
        res = epoch(variant, W_epochs[epoch_i], S_epochs[epoch_i], B_state, cfg, W_prev=W_prev)
        B_state = res[state_key(variant)]
        if variant == YUMA2:
            W_prev = res["weight"]
        C_prev = res["server_consensus_weight"]
        Dn.append(res["validator_reward_normalized"])
        Cs.append(C_prev)
        Is.append(res["server_incentive"])
        Bs.append(np.array(B_state, copy=True))
    out = {"Dn": np.stack(Dn), "C": np.stack(Cs), "I": np.stack(Is), "B": np.stack(Bs)}
    if validators is not None:
        out["dividends"] = dividends_per_1000_tao(validators, S_epochs, out["Dn"], cfg)
    return out


def dividends_per_1000_tao(validators, S_epochs, Dn, cfg) -> dict[str, list[float]]:
    """simulation_utils.py:48-49,95-107."""
    units = ((np.asarray(S_epochs, F32) * F32(cfg.total_subnet_stake)).astype(F32) / F32(1000.0)).astype(F32)
    emis = ((F32(cfg.validator_emission_ratio) * np.asarray(Dn, F32)).astype(F32)
            * F32(cfg.total_epoch_emission)).astype(F32)
    out = {v: [] for v in validators}
    for e in range(units.shape[0]):
        for i, v in enumerate(validators):
            su = float(units[e, i])
            out[v].append(float(emis[e, i]) / su if su > 1e-6 else 0.0)
    return out
