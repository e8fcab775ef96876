"""CPU check of the consensus kernel's exact-stake histogram finish.

`k_consensus_w` (yuma_engine.hip) replaces the tail of the reference's
bisection (yumas.py:195-209) by one stake histogram over the bracket's grid
points when every normalised stake is a multiple of 2^-24 totalling <= 1
(DESIGN.md §2). This file restates that algorithm step for step in numpy —
bracket from the fp32 bit patterns, bisection down to 63 grid points, integer
stake-unit histogram, `lo + 1 + #{b in [1, w-1] : F(lo+b) > κ}` — and checks
it against the oracle's plain bisection (oracle.yuma_oracle.consensus) on
exact-stake inputs: random and integer weights, zero rows / columns, ties on
grid points, NaN / ±inf / negative weights, every κ and precision setting the
GPU tests use. The GPU path itself is compared with the bisection bitwise in
tests/test_gpu_parity.py::test_consensus_histogram_finish_equals_bisection.
"""

import zlib

import numpy as np
import pytest

from oracle import yuma_oracle as orc

F32 = np.float32
KHB = 64  # grid points per column histogram (kHB in the kernel)


def _stakes(rng, V):
    s = rng.pareto(1.5, V) + 0.05
    units = np.floor(s / s.sum() * 2**20).astype(np.int64)
    units[0] += 2**20 - units.sum()
    return (units.astype(np.float64) / 2**20).astype(F32)


def hist_consensus(Wn: np.ndarray, S: np.ndarray, kappa: float, iters: int) -> np.ndarray:
    V, M = Wn.shape
    top = 1 << iters
    scale = F32(top)
    u = S.astype(np.float64) * 2**24
    assert np.all(u == np.floor(u)) and u.sum() <= 2**24, "exact-stake inputs only"
    units = u.astype(np.int64)
    ut = int(units.sum())
    kk = int(np.floor(np.float64(F32(kappa)) * 2**24))
    # bracket (kernel: v_max3_i32 / v_min3_i32 on the bit patterns)
    bits = Wn.astype(F32).view(np.int32)
    imax, imin = bits.max(axis=0), bits.min(axis=0)
    nanc = imax > 0x7F800000
    vmax = imax.astype(np.int32).view(F32)
    vmin = np.where(imin > 0, imin.astype(np.int32).view(F32), F32(0.0))
    stot = S.astype(F32).sum(dtype=F32)
    with np.errstate(invalid="ignore", over="ignore"):
        gmax = np.where(vmax > 0, np.minimum(np.ceil(vmax * scale), scale), 0).astype(np.int64)
        gmin = np.where(vmin > 0, np.minimum(np.ceil(vmin * scale), scale + 1), 0).astype(np.int64)
    lo = np.where(gmin >= 2, gmin - 1, 0)
    hi = np.where(gmax < 1, 1, gmax)
    reset = (lo > 0) & (not stot > F32(kappa))
    lo, hi = np.where(reset, 0, lo), np.where(reset, 1, hi)
    over = lo >= top
    lo, hi = np.where(over, top - 1, lo), np.where(over, top, hi)
    hi = np.where(hi <= lo, lo + 1, hi)
    lo, hi = np.where(nanc, 0, lo), np.where(nanc, top, hi)

    def F(k):  # exact stake units above grid point k, per column
        return np.where(Wn > (k / top).astype(F32)[None, :], units[:, None], 0).sum(axis=0)

    while np.any(hi - lo > KHB - 1):
        act = hi - lo > KHB - 1
        mid = (lo + hi) // 2
        up = F(mid) > kk
        lo = np.where(act & up, mid, lo)
        hi = np.where(act & ~up, mid, hi)
    w = hi - lo
    # bins: clamp(ceil(Wn·2^iters) - lo, 0, w); NaN -> 0 (never above a grid point)
    with np.errstate(invalid="ignore"):
        y = np.ceil(Wn.astype(np.float64) * top - lo[None, :])
    y = np.where(np.isnan(y), 0, y)
    b = np.clip(y, 0, w[None, :]).astype(np.int64)
    out = np.empty(M, dtype=np.int64)
    for m in range(M):
        H = np.bincount(b[:, m], weights=units, minlength=KHB).astype(np.int64)
        P = np.cumsum(H)
        cnt = sum(1 for j in range(1, w[m]) if P[j] < ut - kk)
        # the kernel's form: B = #{b in [0, 64) : P(b) < thr}, lo + max(B, 1)
        B = int(np.count_nonzero(P[:KHB] < ut - kk))
        assert max(B, 1) == 1 + cnt
        out[m] = lo[m] + max(B, 1)
    return out.astype(np.float64) / top


def _normalise(W):
    rs = (W.sum(axis=1, dtype=F32) + F32(1e-6)).astype(F32)
    with np.errstate(invalid="ignore", divide="ignore"):
        return (W / rs[:, None]).astype(F32)


@pytest.mark.parametrize("kind", ["uniform", "integer", "ties", "edges", "wide"])
@pytest.mark.parametrize("kappa", [0.3, 0.5, 0.7])
@pytest.mark.parametrize("precision", [1000, 100000, 10000000])
def test_histogram_finish_equals_bisection(kind, kappa, precision):
    rng = np.random.default_rng(zlib.crc32(f"{kind}/{kappa}/{precision}".encode()))
    V, M = 40, 96
    S = _stakes(rng, V)
    if kind == "uniform":
        Wn = _normalise(rng.random((V, M), dtype=F32))
    elif kind == "integer":  # the §8d synthetic shape: integer weights, 10 % zeros
        W = np.floor(rng.random((V, M)) * 4095).astype(F32)
        W[rng.random((V, M)) < 0.1] = 0
        Wn = _normalise(W)
    elif kind == "ties":  # values exactly on grid points of every precision
        Wn = (rng.integers(0, 64, (V, M)) / 64.0).astype(F32)
    elif kind == "edges":
        W = rng.random((V, M), dtype=F32)
        W[:, 0] = 0.0
        W[3, :] = 0.0
        Wn = _normalise(W)
        Wn[5, 7] = np.nan
        Wn[6, 9] = np.inf
        Wn[7, 11] = -np.inf
        Wn[8, 13] = -0.5
        Wn[9, 15] = -0.0
    else:  # brackets far wider than 64 grid points
        Wn = rng.random((V, M), dtype=F32) * F32(0.9) + F32(0.05)
    iters = orc.bisect_iterations(precision)
    ref = orc.consensus(Wn, S, kappa, precision, as_double=True)
    got = hist_consensus(Wn, S, kappa, iters)
    np.testing.assert_array_equal(got, ref)
