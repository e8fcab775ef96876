"""BASELINE.json configs c3 and c4 on the HIP engine, and generic-float
inputs with the summation-order tie window reported (SURVEY §7 hard parts).

c3: a batched sweep of Yuma 4 scenarios drawn from bench.sweep_config's
    bond_alpha x kappa x liquid x (alpha_low, alpha_high) grid at 256 x 4096,
    every scenario against the oracle's run_simulation loop.
c4: the wide subnet 256 x 65536 cut into 8 miner-column shards
    (wide.run_wide_local) against the unsharded engine run and the oracle.
Reference semantics: yumas.py:494-606 (Yuma4), :399-491 (Yuma3),
simulation_utils.py:26-112 (epoch loop)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import yuma_oracle as orc

pytestmark = pytest.mark.gpu

from yuma_simulation._internal import engine, synth, wide  # noqa: E402
from yuma_simulation._internal.yumas import YumaConfig, YumaParams  # noqa: E402

import bench  # noqa: E402  (the c3 grid: bench.sweep_config)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a ROCm GPU"
    engine.load_library()
    yield


def _sweep_ids(n: int) -> list[int]:
    rng = np.random.default_rng(0xC3)
    ids = sorted(int(g) for g in rng.choice(4096, n, replace=False))
    cfgs = [bench.sweep_config(g) for g in ids]
    # both halves of the grid's liquid axis, several kappas and alphas
    assert {c.liquid_alpha for c in cfgs} == {False, True}
    assert len({c.kappa for c in cfgs}) >= 8 and len({c.bond_alpha for c in cfgs}) >= 8
    return ids


def test_c3_sweep_batch_matches_oracle():
    """16 sweep scenarios x 8 epochs at 256 x 4096 in ONE batched engine call
    (bench --config c3's launch), each against the oracle: C exact, the rest
    within 1e-5 (north_star tolerance)."""
    E, N, V, M = 8, 16, 256, 4096
    version = "Yuma 4 (Rhef+relative bonds)"
    ids = _sweep_ids(N)
    cfgs = [bench.sweep_config(g) for g in ids]
    params = [engine.make_params(engine.VARIANT_YUMA4, c) for c in cfgs]
    seed = 0x5EED0003
    W = engine.synth_weights(seed, E, N, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, N, V)).to(W.device)
    res = engine.run(engine.VARIANT_YUMA4, params, W, S, want_hist=True)
    C, Dn, I = res.C.cpu().numpy(), res.Dn.cpu().numpy(), res.I.cpu().numpy()
    Bh = res.B_hist.cpu().numpy()
    Wh, Sh = W.cpu().numpy(), S.cpu().numpy()
    for j, (g, cfg) in enumerate(zip(ids, cfgs)):
        ref = orc.run(version, Wh[:, j], Sh[:, j], cfg)
        tag = f"sweep[{g}] ba={cfg.bond_alpha:.3f} k={cfg.kappa:.3f} liquid={cfg.liquid_alpha}"
        np.testing.assert_array_equal(C[:, j], ref["C"], err_msg=tag)
        assert_close(Dn[:, j], ref["Dn"], what=f"{tag} Dn")
        assert_close(I[:, j], ref["I"], what=f"{tag} I")
        assert_close(Bh[:, j], ref["B"], what=f"{tag} B")


def _shared_vs_replicated_and_oracle(ids: list[int], E: int, oracle_ids: list[int]):
    """The launch `bench.py --config c3` times: every scenario reads ONE W/S
    trajectory (shared_inputs, yuma_run_ex YUMA_RUN_SHARED_INPUTS), no bond
    history. At 256 x 4096 that is the shared-input bond scan
    (launch_bonds_elem: k_bonds_grp<YUMA4, K=4, R=2, P=2>, four scenarios per
    block over one 32-row x 64-miner W tile), the row sums once per input
    epoch and the consensus / quantisation input / rank once per consensus
    class (k_classes). C, Dn, I and B_final must be
    bitwise those of the same run on W and S replicated per scenario (every
    scenario computing its own everything), and each scenario in oracle_ids
    must match the oracle's run_simulation loop (C exact, the rest 1e-5)."""
    V, M = 256, 4096
    version = "Yuma 4 (Rhef+relative bonds)"
    cfgs = [bench.sweep_config(g) for g in ids]
    N = len(ids)
    params = [engine.make_params(engine.VARIANT_YUMA4, c) for c in cfgs]
    classes = bench.consensus_classes(params)
    seed = 0x5EED0003
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
        assert torch.equal(got[k], getattr(b, k)), f"shared-input {k} differs from the replicated run"
    del b
    torch.cuda.empty_cache()
    Wh, Sh = W[:, 0].cpu().numpy(), S[:, 0].cpu().numpy()
    C, Dn, I, Bf = (got[k].cpu().numpy() for k in ("C", "Dn", "I", "B_final"))
    for j in oracle_ids:
        cfg = cfgs[j]
        ref = orc.run(version, Wh, Sh, cfg)
        tag = f"sweep[{ids[j]}] ba={cfg.bond_alpha:.3f} k={cfg.kappa:.3f} liquid={cfg.liquid_alpha}"
        np.testing.assert_array_equal(C[:, j], ref["C"], err_msg=tag)
        assert_close(Dn[:, j], ref["Dn"], what=f"{tag} Dn")
        assert_close(I[:, j], ref["I"], what=f"{tag} I")
        assert_close(Bf[j], ref["B"][-1], what=f"{tag} B_final")
    return classes


def test_c3_bench_path_32_scenarios_four_classes():
    """32 sweep scenarios (4 kappas x 2 liquid x 4 bond
    alphas, alpha pairs from all 8 blocks of the grid) x 8 epochs through the
    shared-input, history-less path; 4 consensus classes of 8; every scenario
    against the oracle."""
    ids = [b + 16 * k + 256 * liq + 512 * ((b + k + liq) % 8)
           for k in (0, 5, 10, 15) for liq in (0, 1) for b in (0, 5, 10, 15)]
    assert len(ids) == 32
    assert _shared_vs_replicated_and_oracle(ids, 8, list(range(32))) == 4


def test_c3_bench_path_rank0_grid():
    """The exact c3 bench workload of rank 0 (grid points 0..511: 16 consensus
    classes of 32 scenarios, both liquid settings) for 4 epochs: bitwise equal
    to the replicated run; one scenario per class (liquid alternating) against
    the oracle."""
    ids = list(range(512))
    oracle_ids = [16 * k + 256 * (k % 2) + (3 * k) % 16 for k in range(16)]
    assert _shared_vs_replicated_and_oracle(ids, 4, oracle_ids) == 16


def test_c4_wide_eight_shards_matches_unsharded_and_oracle():
    """256 x 65536 (1024 tiles of 64 miners) cut into 8 shards: C and the bond
    history bit-equal to the unsharded engine run for 3 epochs; C, Dn and B
    against the oracle for the first 2."""
    E, V, M = 3, 256, 65536
    cfg = YumaConfig()
    params = [engine.make_params(engine.VARIANT_YUMA3, cfg)]
    seed = 0x5EED0004
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V)).to(W.device)
    ref = engine.run(engine.VARIANT_YUMA3, params, W, S, want_hist=True)
    got = wide.run_wide_local(engine.VARIANT_YUMA3, params, W, S, 8, want_hist=True)
    torch.cuda.synchronize()
    assert len(got.C) == 8
    C = torch.cat(got.C, dim=2)
    np.testing.assert_array_equal(C.cpu().numpy(), ref.C.cpu().numpy())
    Bh = torch.cat(got.B_hist, dim=3)
    assert torch.equal(Bh, ref.B_hist)
    assert torch.equal(torch.cat(got.B_final, dim=2), ref.B_final)
    assert_close(got.Dn.cpu().numpy(), ref.Dn.cpu().numpy(), what="Dn sharded vs unsharded")
    assert_close(torch.cat(got.I, dim=2).cpu().numpy(), ref.I.cpu().numpy(), what="I sharded vs unsharded")
    del ref
    o = orc.run("Yuma 3 (Rhef)", W[:2, 0].cpu().numpy(), S[:2, 0].cpu().numpy(), cfg)
    np.testing.assert_array_equal(C[:2, 0].cpu().numpy(), o["C"])
    assert_close(got.Dn[:2, 0].cpu().numpy(), o["Dn"], what="Dn vs oracle")
    assert_close(Bh[:2, 0].cpu().numpy(), o["B"], what="B vs oracle")


def test_c4_bench_launch_without_history():
    """the launch `bench.py --config c4` times —
    engine.run(Yuma 3, want_hist=False) at 256 x 65536, i.e. the history-less
    scan k_bonds_elem<YUMA3, R=1, VEC, P=4, VECI> over 64-miner tiles with
    [slice][tile][V] dividend partials. 3 epochs: C, Dn, I and B_final bitwise
    those of the history run (the wide history scan, [slice][V][tile]
    partials, same summation order); 2 epochs against the oracle: C exact,
    Dn, I and B_final within 1e-5 (yumas.py:452-476)."""
    E, V, M = 3, 256, 65536
    cfg = YumaConfig()
    params = [engine.make_params(engine.VARIANT_YUMA3, cfg)]
    seed = 0x5EED0004
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V)).to(W.device)
    a = engine.run(engine.VARIANT_YUMA3, params, W, S, want_hist=False)
    b = engine.run(engine.VARIANT_YUMA3, params, W, S, want_hist=True)
    torch.cuda.synchronize()
    for k in ("C", "Dn", "I", "B_final"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    assert torch.equal(a.B_final[0], b.B_hist[-1, 0])
    del a, b
    a2 = engine.run(engine.VARIANT_YUMA3, params, W[:2].contiguous(), S[:2].contiguous(), want_hist=False)
    torch.cuda.synchronize()
    o = orc.run("Yuma 3 (Rhef)", W[:2, 0].cpu().numpy(), S[:2, 0].cpu().numpy(), cfg)
    np.testing.assert_array_equal(a2.C[:, 0].cpu().numpy(), o["C"])
    assert_close(a2.Dn[:, 0].cpu().numpy(), o["Dn"], what="Dn vs oracle")
    assert_close(a2.I[:, 0].cpu().numpy(), o["I"], what="I vs oracle")
    assert_close(a2.B_final[0].cpu().numpy(), o["B"][-1], what="B_final vs oracle")


def _tie_report(C_gpu, C_ref, W, S, cfg, as_double=False):
    """(mismatched columns outside the tie window, tie-window size, mismatches inside)."""
    flags = orc.tie_columns(W, S, cfg.kappa, cfg.consensus_precision, as_double)
    bad = C_gpu != C_ref
    return int((bad & ~flags).sum()), int(flags.sum()), int((bad & flags).sum())


@pytest.mark.parametrize("variant,version", [(engine.VARIANT_YUMA3, "Yuma 3 (Rhef)"),
                                             (engine.VARIANT_RUST, "Yuma 0 (subtensor)")])
def test_random_float_epochs_tie_window(variant, version, record_property):
    """8 epochs of uniform-random fp32 weights at 256 x 4096. Summation order
    (torch's, numpy's, the engine's DPP trees) can only move consensus on
    columns inside the tie window (oracle.tie_columns); everywhere else C is
    bit-equal to the oracle, and while no column has moved, Dn / I / B are
    within 1e-5. The window size and the in-window flips are reported; at
    this fixed seed (a deterministic run) no column may flip, so the value
    checks always run (never skip them)."""
    E, V, M = 8, 256, 4096
    rng = np.random.default_rng(0x7E5 + variant)
    W = rng.random((E, 1, V, M), dtype=np.float32)
    W *= rng.random((E, 1, V, M), dtype=np.float32) < 0.5  # sparse rows, as real subnets
    S = rng.random((E, 1, V), dtype=np.float32)
    cfg = YumaConfig()
    res = engine.run(variant, [engine.make_params(variant, cfg)], torch.from_numpy(W), torch.from_numpy(S),
                     want_hist=True)
    ref = orc.run(version, W[:, 0], S[:, 0], cfg)
    C = res.C[:, 0].cpu().numpy()
    total_win = total_flip = 0
    for e in range(E):
        outside, win, inside = _tie_report(C[e], ref["C"][e], W[e, 0], S[e, 0], cfg, variant == engine.VARIANT_RUST)
        assert outside == 0, f"epoch {e}: {outside} columns differ outside the tie window"
        total_win += win
        total_flip += inside
    record_property("tie_window_columns", total_win)
    record_property("tie_window_flips", total_flip)
    print(f"\n{version}: tie window {total_win} of {E * M} columns, {total_flip} flipped")
    assert total_flip == 0, f"{total_flip} tie-window columns flipped at this seed"
    assert_close(res.Dn[:, 0].cpu().numpy(), ref["Dn"], what="Dn")
    assert_close(res.I[:, 0].cpu().numpy(), ref["I"], what="I")
    assert_close(res.B_hist[:, 0].cpu().numpy(), ref["B"], what="B")


@pytest.mark.parametrize("V,M", [(256, 4096), (200, 1000)])
def test_paired_and_wave_consensus_agree_on_float_stakes(V, M, record_property):
    """runs without the prerank P take the paired consensus kernel
    (k_consensus_p: each wave pair's stake sums go h0 + h1), runs with P the
    wave-owned one (k_consensus_w, another addition order). On generic float
    stakes (no exact-stake histogram finish: both bisect) their C may differ
    only in columns inside the oracle's tie window; at this seed none flips,
    so C is bitwise equal. Against the oracle (numpy's summation order) C is
    equal outside the tie window, and Dn within 1e-5 on every epoch whose
    columns all agree (yumas.py:195-211)."""
    E = 6
    rng = np.random.default_rng(0xC0 + V)
    W = rng.random((E, 1, V, M), dtype=np.float32)
    W *= rng.random((E, 1, V, M), dtype=np.float32) < 0.6
    S = rng.random((E, 1, V), dtype=np.float32) + np.float32(1e-3)
    cfg = YumaConfig()
    params = [engine.make_params(engine.VARIANT_YUMA3, cfg)]
    a = engine.run(engine.VARIANT_YUMA3, params, torch.from_numpy(W), torch.from_numpy(S))
    b = engine.run(engine.VARIANT_YUMA3, params, torch.from_numpy(W), torch.from_numpy(S), want=("P",))
    torch.cuda.synchronize()
    Ca, Cb = a.C[:, 0].cpu().numpy(), b.C[:, 0].cpu().numpy()
    ref = orc.run("Yuma 3 (Rhef)", W[:, 0], S[:, 0], cfg)
    win = flips = checked = 0
    Dn = a.Dn[:, 0].cpu().numpy()
    for e in range(E):
        flags = orc.tie_columns(W[e, 0], S[e, 0], cfg.kappa, cfg.consensus_precision)
        win += int(flags.sum())
        assert not ((Ca[e] != Cb[e]) & ~flags).any(), f"epoch {e}: kernels differ outside the tie window"
        out, _, inside = _tie_report(Ca[e], ref["C"][e], W[e, 0], S[e, 0], cfg)
        assert out == 0, f"epoch {e}: {out} columns differ from the oracle outside the tie window"
        flips += inside
        if flips == 0:  # no flipped column so far, none carried by the bond state
            assert_close(Dn[e], ref["Dn"][e], what=f"Dn[{e}]")
            checked += 1
    record_property("tie_window_columns", win)
    record_property("tie_window_flips_vs_oracle", flips)
    print(f"\n{V}x{M}: tie window {win} columns, {flips} flipped against the oracle, Dn checked on {checked} epochs")
    np.testing.assert_array_equal(Ca, Cb)
    assert checked >= 1


def test_wide_float_weights_against_oracle():
    """miner-column shards on generic float weights. The shards'
    row-sum partials add up in shard order, not the unsharded chunk order, so
    bit-equality with the unsharded run is not claimed; against the oracle C
    is exact outside the tie window and the rest within 1e-5."""
    E, V, M = 4, 64, 1000
    rng = np.random.default_rng(0x51DE)
    W = rng.random((E, 1, V, M), dtype=np.float32)
    S = rng.random((E, 1, V), dtype=np.float32)
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=True))
    params = [engine.make_params(engine.VARIANT_YUMA4, cfg)]
    got = wide.run_wide_local(engine.VARIANT_YUMA4, params, torch.from_numpy(W), torch.from_numpy(S), 3,
                              want_hist=True)
    torch.cuda.synchronize()
    ref = orc.run("Yuma 4 (Rhef+relative bonds) - liquid alpha on", W[:, 0], S[:, 0], cfg)
    C = torch.cat(got.C, dim=2)[:, 0].cpu().numpy()
    flips = 0
    for e in range(E):
        outside, _, inside = _tie_report(C[e], ref["C"][e], W[e, 0], S[e, 0], cfg)
        assert outside == 0, f"epoch {e}"
        flips += inside
    print(f"\nwide float weights: {flips} tie-window columns flipped")
    assert flips == 0, f"{flips} tie-window columns flipped at this seed"
    assert_close(got.Dn[:, 0].cpu().numpy(), ref["Dn"], what="Dn")
    assert_close(torch.cat(got.B_hist, dim=3)[:, 0].cpu().numpy(), ref["B"], what="B")


@pytest.mark.parametrize("variant,extra,reset,chunk,want,N", [
    (engine.VARIANT_YUMA4, {"liquid_alpha": True}, None, 0, ("R", "D"), 6),
    (engine.VARIANT_YUMA3, {}, (3, 5), 4, ("R", "D"), 6),
    (engine.VARIANT_YUMA3, {}, None, 0, ("R", "D", "T", "Tv"), 6),
    (engine.VARIANT_YUMA2, {"liquid_alpha": True}, None, 3, ("R", "D"), 6),
    (engine.VARIANT_RUST, {}, None, 0, ("R", "D"), 6),
    (engine.VARIANT_YUMA1, {"bond_penalty": 0.5}, None, 5, ("R", "D"), 6),
    # k_bonds_grp's fixed-alpha operand (p_corr) with the history
    # stream, and its conditional reset reading the previous slice's C of
    # scenario n0 + k; odd N leaves the last block one scenario (nk < K)
    (engine.VARIANT_YUMA4, {}, None, 0, ("R", "D"), 7),
    (engine.VARIANT_YUMA4, {}, (4, 7, "zero"), 0, ("R", "D"), 7),
    (engine.VARIANT_YUMA4, {"liquid_alpha": True}, (2, 7, "zero"), 3, (), 5),
    # liquid alpha on odd scenarios only: classes whose representative is not
    # liquid still select quantiles once for their liquid members
    (engine.VARIANT_YUMA4, {"liquid_odd": True}, None, 0, ("R", "D"), 6),
    # the column-normalised strip scan (k_bonds_cn: V > 64), padded rows
    (engine.VARIANT_RUST, {"liquid_alpha": True}, None, 4, ("R", "D"), (5, 200)),
    (engine.VARIANT_YUMA1, {}, None, 0, ("R", "D", "T", "Tv"), (6, 130)),
    (engine.VARIANT_YUMA2, {}, None, 3, ("R", "D"), (4, 256)),
    # Yuma 1 run outputs above 64 validators on shared inputs take
    # the rank-class dedup (k_classes with bond_penalty) AND the bond column
    # sums csb / csr of the element-wise scan; a duplicate scenario's scan
    # reads its representative's csb / csr (κ repeats every 3 scenarios, so
    # every class has duplicates). 130 validators: k_rank_s; 1100: above
    # kRegRows, the 256-miner column-block rank k_rank_sw
    (engine.VARIANT_YUMA1, {}, None, 0, ("R", "D"), (6, 130)),
    (engine.VARIANT_YUMA1, {"bond_penalty": 0.5}, None, 4, (), (7, 130)),
    (engine.VARIANT_YUMA1, {"bond_penalty": 0.5}, None, 0, ("R", "D"), (6, 1100)),
    (engine.VARIANT_YUMA1, {"liquid_alpha": True}, None, 3, (), (5, 1100)),
])
def test_shared_input_sweep_equals_replicated(variant, extra, reset, chunk, want, N):
    """yuma_run_ex(YUMA_RUN_SHARED_INPUTS): N scenarios reading ONE W/S
    trajectory ([E,1,V,M]) give bitwise the results of the same run on W and S
    replicated per scenario — consensus, bonds and their history, dividends,
    incentive — with resets, chunking and Yuma2's W_prev; and scenario 0
    matches the oracle (c3's sweep over one subnet). κ repeats
    across scenarios (three consensus classes of two, k_classes: the second of
    each takes the first's consensus, quantisation input and rank); with P / T
    / T_v requested every scenario computes its own."""
    E, V, M = 10, 64, 512
    if isinstance(N, tuple):
        N, V = N
    seed = 0x5EED0003
    W1 = engine.synth_weights(seed, E, 1, V, M)
    S1 = torch.from_numpy(synth.stakes(seed, E, 1, V, period=3)).to(W1.device)
    zero_reset = reset is not None and len(reset) > 2
    if zero_reset:
        # an all-zero miner column quantises to C = 0, so the conditional
        # reset (simulation_utils.py:79-85) fires the epoch after
        W1[reset[0] - 1, ..., reset[1]] = 0.0
    cfgs = []
    for i in range(N):
        sim = {k: v for k, v in extra.items() if k in ("bond_penalty",)}
        prm = {k: v for k, v in extra.items() if k not in ("bond_penalty", "liquid_odd")}
        if extra.get("liquid_odd"):
            prm["liquid_alpha"] = i % 2 == 1
        cfgs.append(YumaConfig(simulation=bench_sim(kappa=0.3 + 0.08 * (i % 3), **sim),
                               yuma_params=YumaParams(bond_alpha=0.05 + 0.05 * i, **prm)))
    kw = {}
    if reset is not None:
        mode = engine.RESET_IF_ZERO_CONSENSUS if zero_reset else engine.RESET_ALWAYS
        kw = {"reset_mode": mode, "reset_epoch": reset[0], "reset_index": reset[1],
              "n_miners": M, "n_epochs": E}
    params = [engine.make_params(variant, c, **kw) for c in cfgs]
    a = engine.run(variant, params, W1, S1, want_hist=True, want=want, chunk_epochs=chunk,
                   shared_inputs=True)
    b = engine.run(variant, params, W1.expand(E, N, V, M).contiguous(), S1.expand(E, N, V).contiguous(),
                   want_hist=True, want=want, chunk_epochs=chunk)
    torch.cuda.synchronize()
    for x, y in ((a.C, b.C), (a.Dn, b.Dn), (a.I, b.I), (a.B_hist, b.B_hist), (a.B_final, b.B_final)):
        assert torch.equal(x, y)
    for k in want:
        assert torch.equal(a.extra[k], b.extra[k]), k
    version = {engine.VARIANT_RUST: "Yuma 0 (subtensor)", engine.VARIANT_YUMA1: "Yuma 1 (paper)",
               engine.VARIANT_YUMA2: "Yuma 2 (Adrian-Fish)", engine.VARIANT_YUMA3: "Yuma 3 (Rhef)",
               engine.VARIANT_YUMA4: "Yuma 4 (Rhef+relative bonds)"}[variant]
    if zero_reset:
        assert (a.C[reset[0] - 1, :, reset[1]] == 0).all()
    if reset is None or zero_reset:
        rk = {}
        if zero_reset:
            rk = {"reset_epoch": reset[0], "reset_index": reset[1]}
        ref = orc.run(version, W1[:, 0].cpu().numpy(), S1[:, 0].cpu().numpy(), cfgs[0], **rk)
        np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"])
        assert_close(a.Dn[:, 0].cpu().numpy(), ref["Dn"], what="shared sweep Dn vs oracle")
        assert_close(a.B_hist[:, 0].cpu().numpy(), ref["B"], what="shared sweep B vs oracle")
        if zero_reset:  # the reset fired: without it the column's bonds differ
            ref0 = orc.run(version, W1[:, 0].cpu().numpy(), S1[:, 0].cpu().numpy(), cfgs[0])
            e, j = reset[0], reset[1]
            assert not np.allclose(ref0["B"][e][:, j], ref["B"][e][:, j])
            np.testing.assert_array_equal(ref["B"][e - 1][:, j] > 0, ref0["B"][e - 1][:, j] > 0)


def bench_sim(**kw):
    from yuma_simulation._internal.yumas import SimulationHyperparameters

    return SimulationHyperparameters(**kw)


@pytest.mark.parametrize("case", ["negative_weight", "alpha_above_one", "state_above_one", "liquid_negative_weight"])
def test_sweep_bounded_update_and_its_fallbacks(case):
    """The sweep scan drops Yuma 4's two clamps when a wave's bond state starts
    in [0, 1], every bond_alpha and 1 - bond_alpha are in [0, 1] and its rows
    carry no negative weight (grp_scan BND, yumas.py:574-586); otherwise it
    keeps them. Each case breaks one condition for part of the grid and must
    still give bitwise the replicated run (k_bonds_elem, always clamped):
    a negative weight in one row at one epoch, bond_alpha = 1.5 for some
    scenarios, a starting bond state above 1, and the negative weight again
    with liquid alpha on half of the grid (mixed blocks). (A liquid alpha
    outside (0, 1) is a ValueError before any run, as in the reference.)"""
    E, N, V, M = 9, 8, 64, 512
    seed = 0x5EEDB0D
    W1 = engine.synth_weights(seed, E, 1, V, M)
    S1 = torch.from_numpy(synth.stakes(seed, E, 1, V, period=4)).to(W1.device)
    cfgs = []
    for i in range(N):
        ba = 0.05 + 0.07 * i
        if case == "alpha_above_one" and i % 3 == 1:
            ba = 1.5
        liq = case == "liquid_negative_weight" and i % 2 == 0
        yp = YumaParams(bond_alpha=ba, liquid_alpha=liq)
        cfgs.append(YumaConfig(simulation=bench_sim(kappa=0.35 + 0.1 * (i % 2)), yuma_params=yp))
    if case in ("negative_weight", "liquid_negative_weight"):
        W1[4, 0, 17, 100] = -3.0
    B0 = None
    if case == "state_above_one":
        B0 = torch.rand(N, V, M, device=W1.device)
        B0[:, 5, :] += 1.0
    params = [engine.make_params(engine.VARIANT_YUMA4, c) for c in cfgs]
    a = engine.run(engine.VARIANT_YUMA4, params, W1, S1, B0, want_hist=False, shared_inputs=True)
    b = engine.run(engine.VARIANT_YUMA4, params, W1.expand(E, N, V, M).contiguous(), S1.expand(E, N, V).contiguous(),
                   B0, want_hist=False)
    torch.cuda.synchronize()
    for k in ("C", "Dn", "I", "B_final"):
        assert torch.equal(getattr(a, k), getattr(b, k)), f"{case}: {k} differs from the replicated run"
    if case != "state_above_one":
        ref = orc.run("Yuma 4 (Rhef+relative bonds)", W1[:, 0].cpu().numpy(), S1[:, 0].cpu().numpy(), cfgs[1])
        np.testing.assert_array_equal(a.C[:, 1].cpu().numpy(), ref["C"])
        assert_close(a.Dn[:, 1].cpu().numpy(), ref["Dn"], what=f"{case} Dn")
        assert_close(a.B_final[1].cpu().numpy(), ref["B"][-1], what=f"{case} B_final")


@pytest.mark.parametrize("V,M,variant", [(12, 100, engine.VARIANT_YUMA4), (10, 99, engine.VARIANT_YUMA3),
                                         (40, 200, engine.VARIANT_YUMA1), (40, 130, engine.VARIANT_RUST)])
def test_shared_input_multiclass_small_shapes(V, M, variant):
    """The multi-class consensus / rank of shared-input sweeps (k_class_list,
    k_consensus_mc, k_rank_mc) at the wave-owned row forms R = 1 (<= 16
    validators) and R = 4 (<= 64), a last tile cut short (M not a multiple of
    64) and M not a multiple of 4 (the scalar loads): bitwise the replicated
    run, scenario 0 against the oracle."""
    E, N = 7, 9
    seed = 0x5EED0C1A + V + M
    W1 = engine.synth_weights(seed, E, 1, V, M)
    S1 = torch.from_numpy(synth.stakes(seed, E, 1, V, period=3)).to(W1.device)
    cfgs = [YumaConfig(simulation=bench_sim(kappa=0.3 + 0.1 * (i % 3)),
                       yuma_params=YumaParams(bond_alpha=0.05 + 0.03 * i, liquid_alpha=i % 2 == 1))
            for i in range(N)]
    params = [engine.make_params(variant, c) for c in cfgs]
    a = engine.run(variant, params, W1, S1, want_hist=True, shared_inputs=True)
    b = engine.run(variant, params, W1.expand(E, N, V, M).contiguous(), S1.expand(E, N, V).contiguous(),
                   want_hist=True)
    torch.cuda.synchronize()
    for k in ("C", "Dn", "I", "B_hist", "B_final"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    version = {engine.VARIANT_RUST: "Yuma 0 (subtensor)", engine.VARIANT_YUMA1: "Yuma 1 (paper)",
               engine.VARIANT_YUMA3: "Yuma 3 (Rhef)", engine.VARIANT_YUMA4: "Yuma 4 (Rhef+relative bonds)"}[variant]
    ref = orc.run(version, W1[:, 0].cpu().numpy(), S1[:, 0].cpu().numpy(), cfgs[0])
    np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"])
    assert_close(a.Dn[:, 0].cpu().numpy(), ref["Dn"], what="Dn")
    assert_close(a.B_hist[:, 0].cpu().numpy(), ref["B"], what="B")
