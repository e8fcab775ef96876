"""Deterministic synthetic subnet inputs.

The reference ships no large inputs; benchmarks and parity tests at
256 validators x 4096 miners use this generator instead. It is integer-only so
the numpy version here and the HIP kernel ``k_synth`` (csrc/yuma_engine.hip)
produce bit-identical weights.

Design ("exactness-friendly", so CPU and GPU make identical discrete
decisions whatever their reduction order):
  * weights are integer-valued fp32 with every row sum < 2**24, so
    ``W.sum(dim=1)`` is exact in any order and ``rs + 1e-6 == rs`` once the
    row sum is >= 32 (yumas.py:186);
  * stakes are integers summing to exactly 2**20, so ``S / S.sum()`` is dyadic
    and every masked stake sum of the consensus bisection (yumas.py:203-204)
    is exact;
  * a per-miner quality factor spreads the consensus over many quantisation
    levels so the liquid-alpha quantiles (yumas.py:237-246) do not tie.
"""

from __future__ import annotations

import numpy as np

MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)
TAG_WEIGHT = np.uint64(1 << 63)
TAG_ZERO = np.uint64(1 << 62)
TAG_QUALITY = np.uint64(1 << 61)
TAG_STAKE = np.uint64(1 << 60)
SCENARIO_STRIDE = 0x1000003
ZERO_THRESHOLD = 1677722  # ~0.1 * 2**24: probability that a weight is zeroed
STAKE_TOTAL = 1 << 20


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _hash3(seed, a, b, c) -> np.ndarray:
    seed = np.uint64(seed)
    return _splitmix64(_splitmix64(_splitmix64(seed ^ np.asarray(a, np.uint64)) ^ np.asarray(b, np.uint64)) ^ np.asarray(c, np.uint64))


def _u24(h: np.ndarray) -> np.ndarray:
    return h >> np.uint64(40)


def scenario_seed(seed: int, n: int) -> np.uint64:
    with np.errstate(over="ignore"):
        return np.uint64((int(seed) + SCENARIO_STRIDE * int(n)) & 0xFFFFFFFFFFFFFFFF)


def max_weight(M: int) -> int:
    return (2**24 - 1) // M


def weights(seed: int, E: int, N: int, V: int, M: int, t0: int = 0) -> np.ndarray:
    """W[e, n, v, m] for epochs t0..t0+E-1 (float32, integer-valued)."""
    out = np.empty((E, N, V, M), dtype=np.float32)
    wmax = np.uint64(max_weight(M))
    m = np.arange(M, dtype=np.uint64)[None, :]
    v = np.arange(V, dtype=np.uint64)[:, None]
    for n in range(N):
        sd = scenario_seed(seed, n)
        qa = _u24(_hash3(sd, TAG_QUALITY, np.uint64(0), m))
        Q = np.uint64(1 << 22) + ((np.uint64(3) * qa) >> np.uint64(2))
        for e in range(E):
            t = np.uint64(t0 + e)
            ua = _u24(_hash3(sd, TAG_WEIGHT | t, v, m))
            F = (np.uint64(3 * (1 << 24)) + np.uint64(4) * ua) // np.uint64(5)
            w = (Q * F) >> np.uint64(24)
            w = np.minimum(w, np.uint64(1 << 24))
            val = (w * wmax) >> np.uint64(24)
            z = _u24(_hash3(sd, TAG_ZERO | t, v, m))
            val = np.where(z < np.uint64(ZERO_THRESHOLD), np.uint64(0), val)
            out[e, n] = val.astype(np.float32)
    return out


def stakes(seed: int, E: int, N: int, V: int, t0: int = 0, period: int = 100) -> np.ndarray:
    """S[e, n, v]: Pareto-like integer stakes summing to exactly 2**20, redrawn
    every `period` epochs."""
    out = np.empty((E, N, V), dtype=np.float32)
    v = np.arange(V, dtype=np.uint64)
    for n in range(N):
        sd = scenario_seed(seed, n)
        cache: dict[int, np.ndarray] = {}
        for e in range(E):
            block = (t0 + e) // period
            if block not in cache:
                u = _u24(_hash3(sd, TAG_STAKE | np.uint64(block), v, np.uint64(0))).astype(np.float64) / 2.0**24
                raw = (1.0 - u) ** (-2.0 / 3.0)
                share = raw / raw.sum() * STAKE_TOTAL
                s = np.floor(share).astype(np.int64)
                rem = STAKE_TOTAL - int(s.sum())
                frac = share - s
                order = np.lexsort((np.arange(V), -frac))  # largest fraction first, then index
                s[order[:rem]] += 1
                cache[block] = s.astype(np.float32)
            out[e, n] = cache[block]
    return out


def random_float_inputs(seed: int, E: int, V: int, M: int):
    """Generic (not exactness-friendly) inputs: uniform floats, the stress set
    of SURVEY §8d. Returned as float32 numpy arrays [E, V, M], [E, V]."""
    rng = np.random.default_rng(seed)
    W = rng.random((E, V, M), dtype=np.float32)
    S = rng.random((E, V), dtype=np.float32)
    return W, S
