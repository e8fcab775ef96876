"""Bench-length trajectories on the HIP engine.

The bench lines time whole trajectories (c2: 1000 epochs in one chunk; c3: 32
epochs; c4: 100 epochs without the bond history). These tests run those exact
launches at their full length and pin them:
  * c2: the captured 1000-epoch hipGraph (the timed step) is bitwise equal to
    the same run cut into 64-epoch chunks, and its last two epochs equal the
    oracle resumed from the engine's own bond state at epoch 997
    (yumas.py:452-476, simulation_utils.py:44-110);
  * the history-less scan parks its quad partials in LDS and flushes them when
    256 epochs fill the buffer (k_bonds_elem DP_QTE): 300-epoch runs, one chunk
    and an odd chunk, bitwise equal to the history run, at c2's shape (one row
    per lane) and at a c4-width grid (two rows per lane);
  * c3: the shared-input sweep for its full 32 epochs, bitwise equal to the
    replicated run.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import yuma_oracle as orc

pytestmark = pytest.mark.gpu

from yuma_simulation._internal import engine, synth  # noqa: E402
from yuma_simulation._internal.yumas import YumaConfig, YumaParams  # noqa: E402

import bench  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a ROCm GPU"
    engine.load_library()
    yield
    torch.cuda.empty_cache()


def _equal_fields(a, b, fields, tag=""):
    for k in fields:
        x, y = getattr(a, k), getattr(b, k)
        assert torch.equal(x, y), f"{tag} {k} differs"


def test_c2_timed_launch_full_trajectory():
    """c2's timed step: 256 x 4096 x 1000 epochs, Yuma 3, bond history, one
    chunk, replayed from the captured hipGraph (bench.engine_line). Bitwise
    equal to the 64-epoch-chunk run; epochs 998-999 against the oracle resumed
    from the engine's B_hist[997]: C exact, Dn / I / B within 1e-5."""
    E, V, M = 1000, 256, 4096
    seed = bench.input_seed("c2", 0x5EED0002, 0)
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V)).to(W.device)
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=False))
    params = [engine.make_params(engine.VARIANT_YUMA3, cfg)]
    g = engine.RunGraph(engine.VARIANT_YUMA3, params, W, S, want_hist=True)
    a = g.launch()
    b = engine.run(engine.VARIANT_YUMA3, params, W, S, want_hist=True, chunk_epochs=64)
    torch.cuda.synchronize()
    _equal_fields(a, b, ("B_hist", "Dn", "C", "I", "B_final"), "c2 graph vs 64-epoch chunks")
    assert torch.equal(a.B_final[0], a.B_hist[-1, 0])
    del b
    torch.cuda.empty_cache()
    B = a.B_hist[997, 0].cpu().numpy()
    for t in (998, 999):
        r = orc.epoch("yuma3", W[t, 0].cpu().numpy(), S[t, 0].cpu().numpy(), B, cfg)
        np.testing.assert_array_equal(a.C[t, 0].cpu().numpy(), r["server_consensus_weight"], err_msg=f"C[{t}]")
        assert_close(a.Dn[t, 0].cpu().numpy(), r["validator_reward_normalized"], what=f"Dn[{t}]")
        assert_close(a.I[t, 0].cpu().numpy(), r["server_incentive"], what=f"I[{t}]")
        assert_close(a.B_hist[t, 0].cpu().numpy(), r["validator_bonds"], what=f"B[{t}]")
        B = r["validator_bonds"]
    g.close()


@pytest.mark.parametrize("V,M,N", [(256, 4096, 1), (256, 32768, 1)])
def test_history_less_scan_past_the_lds_flush(V, M, N):
    """300 epochs without the bond history: the history-less scan
    (k_bonds_elem, DP_QTE quad partials parked in LDS) flushes its 256-epoch
    buffer mid-launch (yuma_engine.hip kQBuf). One chunk and a 37-epoch chunk
    (not a multiple of 16: the epoch-minor partial runs start mid-row) must
    give C / Dn / I / B_final bitwise those of the history run. 256 x 4096 is
    the one-row-per-lane form (c2 --no-history), 256 x 32768 fills the grid
    with 4096 two-row blocks (c4's form)."""
    E = 300
    seed = 0x5EED0004 + M
    W = engine.synth_weights(seed, E, N, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, N, V, period=37)).to(W.device)
    params = [engine.make_params(engine.VARIANT_YUMA3, YumaConfig())] * N
    ref = engine.run(engine.VARIANT_YUMA3, params, W, S, want_hist=True)
    torch.cuda.synchronize()
    ref_keep = {k: getattr(ref, k) for k in ("C", "Dn", "I", "B_final")}
    last = ref.B_hist[-1].clone()
    del ref
    torch.cuda.empty_cache()
    for chunk in (0, 37):
        a = engine.run(engine.VARIANT_YUMA3, params, W, S, want_hist=False, chunk_epochs=chunk)
        torch.cuda.synchronize()
        for k, v in ref_keep.items():
            assert torch.equal(getattr(a, k), v), f"{V}x{M} chunk={chunk}: {k} differs from the history run"
        assert torch.equal(a.B_final, last)
        del a


def test_history_less_yuma4_liquid_past_the_lds_flush():
    """The same flush with Yuma 4 liquid alpha (the per-miner bond_alpha
    operand of the scan) at 128 x 4096, 290 epochs."""
    E, V, M = 290, 128, 4096
    W = engine.synth_weights(0x5EED0042, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(0x5EED0042, E, 1, V, period=50)).to(W.device)
    params = [engine.make_params(engine.VARIANT_YUMA4, YumaConfig(yuma_params=YumaParams(liquid_alpha=True)))]
    a = engine.run(engine.VARIANT_YUMA4, params, W, S, want_hist=False)
    b = engine.run(engine.VARIANT_YUMA4, params, W, S, want_hist=True)
    torch.cuda.synchronize()
    _equal_fields(a, b, ("C", "Dn", "I", "B_final"), "Yuma 4 liquid 290 epochs")


def test_c3_full_trajectory_subset():
    """c3's launch for its full 32 epochs (shared inputs, no history) on 64
    scenarios of rank 0's grid (4 consensus classes, both liquid settings):
    C, Dn, I, B_final bitwise those of the replicated run; one scenario per
    class against the oracle's last epoch."""
    E, V, M = 32, 256, 4096
    ids = [16 * k + 256 * liq + b for k in (0, 5, 10, 15) for liq in (0, 1) for b in range(8)]
    assert len(ids) == 64
    cfgs = [bench.sweep_config(g) for g in ids]
    params = [engine.make_params(engine.VARIANT_YUMA4, c) for c in cfgs]
    assert bench.consensus_classes(params) == 4
    N = len(ids)
    seed = bench.input_seed("c3", 0x5EED0003, 0)
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V)).to(W.device)
    a = engine.run(engine.VARIANT_YUMA4, params, W, S, want_hist=False, shared_inputs=True)
    torch.cuda.synchronize()
    got = {k: getattr(a, k).clone() for k in ("C", "Dn", "I", "B_final")}
    del a
    b = engine.run(engine.VARIANT_YUMA4, params, W.expand(E, N, V, M).contiguous(),
                   S.expand(E, N, V).contiguous(), want_hist=False)
    torch.cuda.synchronize()
    for k in got:
        assert torch.equal(got[k], getattr(b, k)), f"c3 32-epoch shared-input {k} differs from the replicated run"
    del b
    torch.cuda.empty_cache()
    Wh, Sh = W[:, 0].cpu().numpy(), S[:, 0].cpu().numpy()
    for j in (0, 41):
        ref = orc.run("Yuma 4 (Rhef+relative bonds)", Wh, Sh, cfgs[j])
        tag = f"sweep[{ids[j]}]"
        np.testing.assert_array_equal(got["C"][:, j].cpu().numpy(), ref["C"], err_msg=tag)
        assert_close(got["Dn"][:, j].cpu().numpy(), ref["Dn"], what=f"{tag} Dn")
        assert_close(got["B_final"][j].cpu().numpy(), ref["B"][-1], what=f"{tag} B_final")


@pytest.mark.parametrize("variant,liquid,N,chunk", [
    (engine.VARIANT_YUMA4, "all", 8, 0),
    (engine.VARIANT_YUMA4, "odd", 7, 23),
    (engine.VARIANT_YUMA3, "none", 6, 0),
])
def test_sweep_scan_past_the_partial_flush(variant, liquid, N, chunk):
    """The sweep scan (k_bonds_grp, shared inputs) parks its dividend
    partials per wave in LDS and writes them every 32 epochs (kGrpDB): 75
    epochs, one chunk and a 23-epoch chunk (flushes that do not start on a
    multiple of 32), every liquid form of a block (all liquid / mixed /
    fixed). Bitwise the results of the replicated run, whose history-less
    scan stores its partials in another layout (the canonical sum is the
    same); scenario 0 against the oracle (yumas.py:452-476, :570-593)."""
    E, V, M = 75, 64, 512
    seed = 0x5EED0075
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V, period=20)).to(W.device)
    cfgs = []
    for i in range(N):
        liq = liquid == "all" or (liquid == "odd" and i % 2 == 1)
        cfgs.append(YumaConfig(simulation=bench_sim(kappa=0.35 + 0.1 * (i % 3)),
                               yuma_params=YumaParams(bond_alpha=0.05 + 0.04 * i, liquid_alpha=liq)))
    params = [engine.make_params(variant, c) for c in cfgs]
    a = engine.run(variant, params, W, S, want_hist=False, chunk_epochs=chunk, shared_inputs=True)
    b = engine.run(variant, params, W.expand(E, N, V, M).contiguous(), S.expand(E, N, V).contiguous(),
                   want_hist=False, chunk_epochs=chunk)
    torch.cuda.synchronize()
    _equal_fields(a, b, ("C", "Dn", "I", "B_final"), f"sweep {liquid} chunk={chunk}")
    version = "Yuma 3 (Rhef)" if variant == engine.VARIANT_YUMA3 else "Yuma 4 (Rhef+relative bonds)"
    ref = orc.run(version, W[:, 0].cpu().numpy(), S[:, 0].cpu().numpy(), cfgs[0])
    np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"])
    assert_close(a.Dn[:, 0].cpu().numpy(), ref["Dn"], what="Dn")
    assert_close(a.B_final[0].cpu().numpy(), ref["B"][-1], what="B_final")


def bench_sim(**kw):
    from yuma_simulation._internal.yumas import SimulationHyperparameters

    return SimulationHyperparameters(**kw)
