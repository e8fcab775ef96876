"""HIP engine parity (gpu marker): the product path — yuma_simulation on
libyuma_hip.so through the C-ABI — against the reference goldens and the CPU
oracle. Bit-exact for discrete outputs (consensus levels, clip decisions,
dividend-sheet CSV text); <= 1e-5 relative for fp32 values."""

import hashlib
import io
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, assert_close
from golden import specs
from oracle import yuma_oracle as orc

pytestmark = pytest.mark.gpu

from yuma_simulation._internal import engine, synth  # noqa: E402
from yuma_simulation._internal import yumas as Y  # noqa: E402
from yuma_simulation._internal.cases import BaseCase, cases  # noqa: E402
from yuma_simulation._internal.simulation_utils import (  # noqa: E402
    SimulationRun,
    generate_total_dividends_table,
    run_simulation,
    run_simulations,
)

FN = {"rust": Y.YumaRust, "yuma1": Y.Yuma, "yuma2": Y.Yuma2, "yuma3": Y.Yuma3, "yuma4": Y.Yuma4}
VARIANT_ID = {"rust": engine.VARIANT_RUST, "yuma1": engine.VARIANT_YUMA1, "yuma2": engine.VARIANT_YUMA2,
              "yuma3": engine.VARIANT_YUMA3, "yuma4": engine.VARIANT_YUMA4}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a ROCm GPU"
    engine.load_library()  # fails loudly if the HIP library is missing
    yield


def config_from(spec):
    sim, par = specs.split_spec(spec)
    return Y.YumaConfig(simulation=Y.SimulationHyperparameters(**sim), yuma_params=Y.YumaParams(**par))


def call(variant, W, S, B_old, cfg, W_prev=None):
    if variant == "yuma2":
        return FN[variant](W, W_prev, S, B_old, cfg)
    return FN[variant](W, S, B_old, cfg)


def state_of(variant, r):
    return r["validator_bonds"] if variant in ("yuma3", "yuma4") else r["validator_ema_bond"]


def to_np(x):
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


# ---------------------------------------------------------------------------
# dividend sheet (config 5) and the built-in cases (config 1)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("bi", range(4))
def test_sheet_csv_byte_identical(bi):
    """generate_total_dividends_table -> CSV text equals the reference's."""
    with open(os.path.join(GOLDEN, "sheet.json")) as f:
        meta = json.load(f)
    beta = specs.BETAS[bi]
    versions = [(v, Y.YumaParams(**p)) for v, p in zip(specs.VERSIONS, specs.SHEET_PARAMS)]
    df = generate_total_dividends_table(cases, versions, Y.SimulationHyperparameters(bond_penalty=beta))
    buf = io.StringIO()
    df.to_csv(buf, index=False, float_format="%.6f")
    name = f"total_dividends_b{beta}.csv"
    assert buf.getvalue() == meta["csv"][name]
    assert hashlib.md5(buf.getvalue().encode()).hexdigest() == meta["csv_md5"][name]


def test_sheet_all_tables_batched_and_scripts(tmp_path):
    """All four sheets from ONE batched call (generate_total_dividends_tables,
    config c5) and the scripts/ generator: the reference's CSV bytes."""
    import sys

    from yuma_simulation._internal.simulation_utils import (
        SHEET_BOND_PENALTIES,
        generate_total_dividends_tables,
        sheet_yuma_versions,
    )

    with open(os.path.join(GOLDEN, "sheet.json")) as f:
        meta = json.load(f)
    frames = generate_total_dividends_tables(
        cases, sheet_yuma_versions(), [Y.SimulationHyperparameters(bond_penalty=b) for b in SHEET_BOND_PENALTIES])
    for beta, df in zip(SHEET_BOND_PENALTIES, frames):
        buf = io.StringIO()
        df.to_csv(buf, index=False, float_format="%.6f")
        assert buf.getvalue() == meta["csv"][f"total_dividends_b{beta}.csv"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from scripts import total_dividends_sheet_generator as gen

    for path in gen.main(str(tmp_path)):
        with open(path, "rb") as f:
            assert hashlib.md5(f.read()).hexdigest() == meta["csv_md5"][os.path.basename(path)]


def test_sheet_totals_with_mixed_reward_scalars():
    """Tables whose hyperparameters differ in the reward scalars (subnet
    stake, emission) land in one engine group with no shared dividend ratio:
    the sheet's totals path then sums each run's own ratios. Every table
    equals the frame built from the runs' per-epoch dividend lists
    (reference simulation_utils.py:341-381 over run_simulation's lists), and
    the same tables one call at a time."""
    from yuma_simulation._internal import simulation_utils as su

    versions = su.sheet_yuma_versions()
    hypers = [Y.SimulationHyperparameters(bond_penalty=0.5),
              Y.SimulationHyperparameters(bond_penalty=0.5, total_subnet_stake=3.5e5),
              Y.SimulationHyperparameters(bond_penalty=0.99, total_epoch_emission=37.0,
                                          validator_emission_ratio=0.3)]
    frames = su.generate_total_dividends_tables(cases, versions, hypers)
    for h, df in zip(hypers, frames):
        runs = su._sheet_runs(cases, versions, h)
        lists = su._sheet_frame(cases, versions, su.run_simulations(runs, want_bonds=False, want_incentives=False))
        one = su.generate_total_dividends_table(cases, versions, h)
        for other in (lists, one):
            assert list(df.columns) == list(other.columns) and df.dtypes.equals(other.dtypes)
            assert df.to_csv(index=False) == other.to_csv(index=False)


def test_sheet_runs_per_epoch(golden):
    """Every (beta, case, version) run: consensus exact, dividends / bonds /
    incentives within tolerance; all 504 runs go through batched launches."""
    g = golden("sheet.npz")
    runs, where = [], []
    for bi, beta in enumerate(specs.BETAS):
        for ci, case in enumerate(cases):
            for vi, version in enumerate(specs.VERSIONS):
                cfg = Y.YumaConfig(simulation=Y.SimulationHyperparameters(bond_penalty=beta),
                                   yuma_params=Y.YumaParams(**specs.SHEET_PARAMS[vi]))
                runs.append(SimulationRun(case, version, cfg))
                where.append((bi, ci, vi))
    results = run_simulations(runs)
    for (bi, ci, vi), (div, bonds, inc) in zip(where, results):
        case = cases[ci]
        tag = f"b{specs.BETAS[bi]} {case.name[:7]} {specs.VERSIONS[vi]}"
        d = np.array([div[v] for v in case.validators]).T
        assert_close(d, g["dividends"][bi, ci, vi], what=tag + " dividends")
        assert_close(np.stack([to_np(b) for b in bonds]), g["bonds"][bi, ci, vi], what=tag + " bonds")
        assert_close(np.stack([to_np(x) for x in inc]), g["incentives"][bi, ci, vi], what=tag + " I")


def test_run_simulation_single_case_matches(golden):
    g = golden("sheet.npz")
    cfg = Y.YumaConfig(simulation=Y.SimulationHyperparameters(bond_penalty=0.99))
    div, bonds, inc = run_simulation(cases[10], "Yuma 1 (paper)", cfg)
    d = np.array([div[v] for v in cases[10].validators]).T
    assert_close(d, g["dividends"][2, 10, 1])
    assert len(bonds) == 40 and bonds[0].device.type == "cpu"


def test_invalid_version_raises():
    with pytest.raises(ValueError, match="Invalid Yuma function."):
        run_simulation(cases[0], "Yuma 7", Y.YumaConfig())


# ---------------------------------------------------------------------------
# single-epoch variant functions (full result dictionaries)
# ---------------------------------------------------------------------------
def _small_cases():
    for iname in ("synth16x64", "rand16x64", "edge3x5"):
        for variant in specs.VARIANTS:
            for cname in specs.CONFIGS:
                if cname.startswith("liquid") and variant == "yuma3":
                    continue
                yield iname, variant, cname


@pytest.mark.parametrize("iname,variant,cname", list(_small_cases()))
def test_epoch_functions_match_reference(golden, iname, variant, cname):
    g = golden("epoch_small.npz")
    cfg = config_from(specs.CONFIGS[cname])
    W0, S0 = torch.from_numpy(g[f"in__{iname}__W0"]), torch.from_numpy(g[f"in__{iname}__S0"])
    W1, S1 = torch.from_numpy(g[f"in__{iname}__W1"]), torch.from_numpy(g[f"in__{iname}__S1"])
    r0 = call(variant, W0, S0, None, cfg)
    prev = r0["weight"] if variant == "yuma2" else None
    r1 = call(variant, W1, S1, state_of(variant, r0).clone(), cfg, W_prev=prev)
    for step, r in (("e0", r0), ("e1", r1)):
        tag = f"out__{iname}__{variant}__{cname}__{step}"
        keys = [k[len(tag) + 2:] for k in g.files if k.startswith(tag + "__") and not k.endswith("__pyfloat")]
        assert list(r) == [k for k in Y.RESULT_KEYS[VARIANT_ID[variant]]]
        assert set(keys) == set(r)
        for k in keys:
            exp = g[f"{tag}__{k}"]
            got = r[k]
            if f"{tag}__{k}__pyfloat" in g.files:
                assert isinstance(got, float), (tag, k)
                assert got == float(exp) or (np.isnan(got) and np.isnan(exp))
                continue
            assert isinstance(got, torch.Tensor) and got.device.type == "cpu", (tag, k)
            if k == "server_consensus_weight":
                np.testing.assert_array_equal(to_np(got), exp, err_msg=f"{tag} {k}")
            elif k == "consensus_clipped_weight":
                # clip decisions: which entries were clipped must be identical,
                # each side judged against its own (normalised) source weights
                src_step = "e0" if variant == "yuma2" else step
                ours = to_np(r["weight"] if variant != "yuma2" or step == "e0" else prev)
                theirs = g[f"out__{iname}__{variant}__{cname}__{src_step}__weight"]
                np.testing.assert_array_equal(to_np(got) < ours, exp < theirs, err_msg=tag)
                assert_close(to_np(got), exp, what=f"{tag} {k}")
            else:
                assert_close(to_np(got), exp, what=f"{tag} {k}")


def test_yuma_alias_without_history():
    W = torch.rand(8, 16)
    S = torch.rand(8)
    r = Y.Yuma(W, S)
    assert r["validator_ema_bond"] is r["validator_bond"]
    assert isinstance(r["bond_alpha"], float) and torch.isnan(r["alpha_a"])


def test_epoch_on_gpu_tensors_stays_on_gpu():
    W = torch.rand(8, 16, device="cuda")
    S = torch.rand(8, device="cuda")
    r = Y.Yuma3(W, S)
    assert r["validator_bonds"].is_cuda


# ---------------------------------------------------------------------------
# multi-epoch runs on synthetic and random inputs (run_simulation path)
# ---------------------------------------------------------------------------
class ArrayCase(BaseCase):
    def __init__(self, W, S, reset_epoch, reset_index):
        names = [f"V{i}" for i in range(W.shape[1])]
        super().__init__(name="synthetic", validators=names, base_validator=names[0], num_epochs=W.shape[0],
                         reset_bonds=True, reset_bonds_index=reset_index, reset_bonds_epoch=reset_epoch)
        self._W = [torch.from_numpy(w.copy()) for w in W]
        self._S = [torch.from_numpy(s.copy()) for s in S]

    @property
    def weights_epochs(self):
        return self._W

    @property
    def stakes_epochs(self):
        return self._S


@pytest.mark.parametrize("sname", ["synth64x512", "rand32x256"])
def test_run_medium_matches_reference(golden, sname):
    g = golden("run_medium.npz")
    W, S = g[f"in__{sname}__W"], g[f"in__{sname}__S"]
    re, ri = (int(x) for x in g[f"in__{sname}__reset"])
    case = ArrayCase(W, S, re, ri)
    for vi, version in enumerate(specs.VERSIONS):
        cfg = Y.YumaConfig(simulation=Y.SimulationHyperparameters(bond_penalty=0.5),
                           yuma_params=Y.YumaParams(**specs.SHEET_PARAMS[vi]))
        div, bonds, inc = run_simulation(case, version, cfg)
        tag = f"out__{sname}__{vi}"
        d = np.array([div[v] for v in case.validators]).T
        assert_close(d, g[f"{tag}__dividends"], what=f"{tag} dividends")
        assert_close(to_np(bonds[-1]), g[f"{tag}__B_last"], what=f"{tag} B_last")
        assert_close(to_np(bonds[0]), g[f"{tag}__B_first"], what=f"{tag} B_first")
        assert_close(np.stack([to_np(b).astype(np.float64).sum(axis=0) for b in bonds]),
                     g[f"{tag}__Bsum_epochs"], what=f"{tag} Bsum")
        assert_close(np.stack([to_np(x) for x in inc]), g[f"{tag}__I"], what=f"{tag} I")


@pytest.mark.parametrize("version", ["Yuma 3.1 (Rhef+reset)", "Yuma 3.2 (Rhef+conditional)",
                                     "Yuma 4 (Rhef+relative bonds)"])
def test_reset_index_python_semantics(version):
    """Negative and None reset_bonds_index as the reference's torch indexing
    reads them (simulation_utils.py:62-88): -k counts from the end; None zeroes
    every column for Yuma 3.1 and raises for Yuma 3.2/4 (M > 1). Checked
    against the oracle, whose numpy indexing has the same semantics."""
    rng = np.random.default_rng(11)
    E, V, M = 8, 16, 40
    W = rng.random((E, V, M), dtype=np.float32)
    W[:, :, 5:9] *= (rng.random((E, V, 4)) < 0.3)  # columns that reach C == 0
    W[3:, :, -3] = 0.0  # the reset column has zero consensus before epoch 4 (fires for 3.2/4)
    S = rng.random((E, V), dtype=np.float32)
    cfg = Y.YumaConfig(simulation=Y.SimulationHyperparameters(bond_penalty=0.5))
    neg = run_simulation(ArrayCase(W, S, 4, -3), version, cfg)
    pos = run_simulation(ArrayCase(W, S, 4, M - 3), version, cfg)
    for a, b in zip(neg[1], pos[1]):
        assert torch.equal(a, b)
    ref = orc.run(version, W, S, cfg, reset_epoch=4, reset_index=-3)
    assert_close(np.stack([to_np(b) for b in neg[1]]), ref["B"], what=f"{version} B (index -3)")
    if version.startswith("Yuma 3.1"):
        allc = run_simulation(ArrayCase(W, S, 4, None), version, cfg)
        ref = orc.run(version, W, S, cfg, reset_epoch=4, reset_index=None)
        assert_close(np.stack([to_np(b) for b in allc[1]]), ref["B"], what="3.1 B (index None)")
        assert not torch.equal(allc[1][4], pos[1][4])
    else:
        with pytest.raises(RuntimeError):
            run_simulation(ArrayCase(W, S, 4, None), version, cfg)
    with pytest.raises(IndexError):
        run_simulation(ArrayCase(W, S, 4, M), version, cfg)


# ---------------------------------------------------------------------------
# BASELINE shape 256 x 4096
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def large_inputs(golden):
    g = golden("large.npz")
    W = synth.weights(specs.LARGE_SEED, 2, 1, 256, 4096)[:, 0]
    S = synth.stakes(specs.LARGE_SEED, 2, 1, 256)[:, 0]
    return g, W, S


@pytest.mark.parametrize("name", list(specs.LARGE_SPECS))
def test_large_epoch_matches_reference(large_inputs, name):
    g, W, S = large_inputs
    variant = name.split("_")[0]
    cfg = config_from(specs.LARGE_SPECS[name])
    r0 = call(variant, torch.from_numpy(W[0]), torch.from_numpy(S[0]), None, cfg)
    prev = r0["weight"] if variant == "yuma2" else None
    r1 = call(variant, torch.from_numpy(W[1]), torch.from_numpy(S[1]), state_of(variant, r0).clone(), cfg,
              W_prev=prev)
    idx = g["sample_idx"]
    for step, r in (("e0", r0), ("e1", r1)):
        tag = f"out__{name}__{step}"
        np.testing.assert_array_equal(to_np(r["server_consensus_weight"]), g[f"{tag}__server_consensus_weight"])
        for k in ("server_incentive", "server_rank", "server_prerank", "validator_reward",
                  "validator_reward_normalized"):
            assert_close(to_np(r[k]), g[f"{tag}__{k}"], what=f"{tag} {k}")
        B = to_np(state_of(variant, r))
        assert_close(B.astype(np.float64).sum(axis=0), g[f"{tag}__B_colsum"], what=f"{tag} Bcol")
        assert_close(B.astype(np.float64).sum(axis=1), g[f"{tag}__B_rowsum"], what=f"{tag} Brow")
        assert_close(B[idx[:, 0], idx[:, 1]], g[f"{tag}__B_sample"], what=f"{tag} Bsample")
        if f"{tag}__bond_alpha" in g.files:
            assert_close(to_np(r["bond_alpha"]), g[f"{tag}__bond_alpha"], what=f"{tag} bond_alpha")


def test_large_random_floats_decisions(golden):
    g = golden("large.npz")
    Wr, Sr = synth.random_float_inputs(int(g["rand__W_seed"]), 1, 256, 4096)
    r = Y.Yuma(torch.from_numpy(Wr[0]), torch.from_numpy(Sr[0]))
    np.testing.assert_array_equal(to_np(r["server_consensus_weight"]), g["rand__server_consensus_weight"])
    assert_close(to_np(r["server_incentive"]), g["rand__server_incentive"])
    assert_close(to_np(r["validator_reward_normalized"]), g["rand__validator_reward_normalized"])


# ---------------------------------------------------------------------------
# engine-level properties at full size (size-independent checks)
# ---------------------------------------------------------------------------
def test_device_synth_matches_numpy():
    for (E, N, V, M) in ((2, 3, 17, 130), (1, 1, 256, 4096)):
        d = engine.synth_weights(0xABCDEF, E, N, V, M, t0=5).cpu().numpy()
        h = synth.weights(0xABCDEF, E, N, V, M, t0=5)
        np.testing.assert_array_equal(d, h)


@pytest.mark.parametrize("variant", list(VARIANT_ID))
def test_multi_epoch_vs_oracle_and_chunk_invariance(variant):
    """12 epochs at 256x4096: engine run == oracle loop (C exact, rest within
    tolerance); and the result is bitwise independent of the chunking (longer
    trajectories from scratch: test_gpu_trajectory.py)."""
    E, V, M = 12, 256, 4096
    W = synth.weights(0x5EED0002, E, 1, V, M)
    S = synth.stakes(0x5EED0002, E, 1, V, period=5)
    cfg = config_from({"liquid_alpha": True} if variant in ("yuma1", "yuma4") else {})
    vid = VARIANT_ID[variant]
    prm = [engine.make_params(vid, cfg)]
    a = engine.run(vid, prm, torch.from_numpy(W), torch.from_numpy(S), want_hist=True, chunk_epochs=E)
    b = engine.run(vid, prm, torch.from_numpy(W), torch.from_numpy(S), want_hist=True, chunk_epochs=5)
    torch.cuda.synchronize()
    assert torch.equal(a.B_hist, b.B_hist) and torch.equal(a.Dn, b.Dn) and torch.equal(a.C, b.C)
    version = {"rust": "Yuma 0 (subtensor)", "yuma1": "Yuma 1 (paper) - liquid alpha on",
               "yuma2": "Yuma 2 (Adrian-Fish)", "yuma3": "Yuma 3 (Rhef)",
               "yuma4": "Yuma 4 (Rhef+relative bonds) - liquid alpha on"}[variant]
    ref = orc.run(version, W[:, 0], S[:, 0], cfg)
    np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"])
    assert_close(a.Dn[:, 0].cpu().numpy(), ref["Dn"], what="Dn")
    assert_close(a.I[:, 0].cpu().numpy(), ref["I"], what="I")
    assert_close(a.B_hist[:, 0].cpu().numpy(), ref["B"], what="B")
    # properties: levels quantised, dividends normalised
    lev = a.C.cpu().numpy() * 65535.0
    assert np.allclose(lev, np.rint(lev), atol=1e-2)
    # Dn = D / (sum D + 1e-6): sums to sum D / (sum D + 1e-6) <= 1 (Yuma4's D is
    # stake-scaled, so the epsilon is visible there)
    tot = a.Dn.sum(dim=-1).cpu().numpy()
    assert np.all(tot <= 1.0 + 1e-5) and np.all(tot > 0.5)


@pytest.mark.parametrize("V,vids", [(64, (engine.VARIANT_YUMA1, engine.VARIANT_YUMA4)),
                                     (160, (engine.VARIANT_RUST, engine.VARIANT_YUMA1, engine.VARIANT_YUMA2)),
                                     (384, (engine.VARIANT_RUST, engine.VARIANT_YUMA1, engine.VARIANT_YUMA2))])
def test_batched_scenarios_equal_individual_runs(V, vids):
    """N scenarios in one launch == each alone (bitwise), params differing.
    V = 160: the column-normalised bond scans with padded rows and a
    half-filled last 16-miner strip; V = 384: 257-512 validators
    on the float4 path (YumaRust's strip scan with four rows per lane)."""
    E, N, M = 6, 5, 1000  # M % 4 == 0 but not a multiple of 64 (nor of 16)
    W = synth.weights(77, E, N, V, M)
    S = synth.stakes(77, E, N, V, period=3)
    cfgs = [config_from({"kappa": 0.3 + 0.1 * n, "liquid_alpha": n % 2 == 1}) for n in range(N)]
    for vid in vids:
        prm = [engine.make_params(vid, c) for c in cfgs]
        full = engine.run(vid, prm, torch.from_numpy(W), torch.from_numpy(S), want_hist=True)
        for n in range(N):
            one = engine.run(vid, [prm[n]], torch.from_numpy(W[:, n:n + 1]), torch.from_numpy(S[:, n:n + 1]),
                             want_hist=True)
            assert torch.equal(full.B_hist[:, n], one.B_hist[:, 0])
            assert torch.equal(full.Dn[:, n], one.Dn[:, 0])


@pytest.mark.parametrize("V,M", [(1, 1), (3, 7), (33, 65), (1024, 96), (300, 130)])
def test_ragged_shapes_vs_oracle(V, M):
    """Odd sizes exercise the scalar (non-float4) path and padded tiles."""
    rng = np.random.default_rng(V * 1000 + M)
    E = 3
    W = rng.random((E, V, M), dtype=np.float32)
    W[:, :, 0] = 0.0
    S = rng.random((E, V), dtype=np.float32) + np.float32(0.01)
    for variant, version in (("yuma1", "Yuma 1 (paper)"), ("rust", "Yuma 0 (subtensor)"),
                             ("yuma3", "Yuma 3 (Rhef)"), ("yuma4", "Yuma 4 (Rhef+relative bonds)"),
                             ("yuma2", "Yuma 2 (Adrian-Fish)")):
        vid = VARIANT_ID[variant]
        cfg = Y.YumaConfig()
        res = engine.run(vid, [engine.make_params(vid, cfg)], torch.from_numpy(W[:, None]),
                         torch.from_numpy(S[:, None]), want_hist=True)
        ref = orc.run(version, W, S, cfg)
        np.testing.assert_array_equal(res.C[:, 0].cpu().numpy(), ref["C"], err_msg=f"{variant} {V}x{M}")
        assert_close(res.Dn[:, 0].cpu().numpy(), ref["Dn"], rtol=1e-4, what=f"{variant} {V}x{M} Dn")
        assert_close(res.B_hist[:, 0].cpu().numpy(), ref["B"], rtol=1e-4, what=f"{variant} {V}x{M} B")


@pytest.mark.parametrize("variant,version,V,M", [
    ("yuma1", "Yuma 1 (paper)", 128, 1024), ("yuma2", "Yuma 2 (Adrian-Fish)", 128, 1024),
    ("yuma3", "Yuma 3 (Rhef)", 128, 1024), ("yuma4", "Yuma 4 (Rhef+relative bonds)", 128, 1024),
    ("yuma3", "Yuma 3 (Rhef)", 256, 32768)])
def test_screened_division_rows_outside_the_screen(variant, version, V, M):
    """The scans that divide W by k_rowsum's screened RN(1 / row sum): the
    Yuma / Yuma2 history scan (the wide layout) and every history-less scan
    (one row per lane at 128 x 1024, two rows per lane at 256 x 32768, c4's
    form); rows with a weight above 2^60 or a nonzero weight below 2^-60 fail
    the screen (NaN reciprocal) and their waves divide by IEEE. Against the
    oracle (yumas.py:217-258, :299-343, :452-476, :570-593) and bitwise
    history against history-less run (one of them divides with the per-row
    guard for Yuma 3 / 4): same C / Dn / I / B_final. Zero and -0 weights too."""
    rng = np.random.default_rng(0x5C4EE + M)
    E = 6
    W = rng.random((E, V, M), dtype=np.float32)
    W[1, 5, 17] = np.float32(3e18)        # > 2^60: row 5 of epoch 1 fails
    W[2, 70, 900] = np.float32(1e-20)     # nonzero below 2^-60
    W[3, 9, :] = 0.0                      # row sum 1e-6 (passes)
    W[3, 9, 3] = np.float32(-0.0)
    W[4, :, 64] = np.float32(-0.0)
    W[5, V - 1, M - 24:] = np.float32(5e20)   # last row, last tile
    S = rng.random((E, V), dtype=np.float32) + np.float32(0.01)
    vid = VARIANT_ID[variant]
    cfg = Y.YumaConfig()
    prm = [engine.make_params(vid, cfg)]
    Wt, St = torch.from_numpy(W[:, None]), torch.from_numpy(S[:, None])
    a = engine.run(vid, prm, Wt, St, want_hist=True)
    b = engine.run(vid, prm, Wt, St, want_hist=False)
    torch.cuda.synchronize()
    for k in ("C", "Dn", "I", "B_final"):
        assert torch.equal(getattr(a, k), getattr(b, k)), f"{variant}: {k} history vs history-less"
    ref = orc.run(version, W, S, cfg)
    # float stakes: C equal to the oracle outside the summation-order tie
    # window (oracle.tie_columns); values compared up to the first epoch with
    # a flipped column (none at 128 x 1024; 256 x 32768 has one in-window flip)
    C = a.C[:, 0].cpu().numpy()
    upto = E
    for e in range(E):
        flags = orc.tie_columns(W[e], S[e], cfg.kappa, cfg.consensus_precision)
        bad = C[e] != ref["C"][e]
        assert not (bad & ~flags).any(), f"{variant} epoch {e}: C differs outside the tie window"
        if bad.any() and upto == E:
            upto = e
    assert upto >= 2, f"{variant}: a tie-window flip already at epoch {upto}"
    assert_close(a.Dn[:upto, 0].cpu().numpy(), ref["Dn"][:upto], what=f"{variant} Dn")
    assert_close(a.I[:upto, 0].cpu().numpy(), ref["I"][:upto], what=f"{variant} I")
    assert_close(a.B_hist[:upto, 0].cpu().numpy(), ref["B"][:upto], what=f"{variant} B")


def test_rejects_too_many_validators():
    big = 2**20 + 1
    with pytest.raises(engine.EngineError):
        engine.run(engine.VARIANT_YUMA3, [engine.make_params(3, Y.YumaConfig())],
                   torch.zeros(1, 1, big, 1), torch.ones(1, 1, big))


def test_deterministic_repeat():
    E, V, M = 4, 256, 4096
    W = engine.synth_weights(3, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(3, E, 1, V)).cuda()
    prm = [engine.make_params(engine.VARIANT_YUMA3, Y.YumaConfig())]
    a = engine.run(engine.VARIANT_YUMA3, prm, W, S, want_hist=True)
    b = engine.run(engine.VARIANT_YUMA3, prm, W, S, want_hist=True)
    torch.cuda.synchronize()
    assert torch.equal(a.B_hist, b.B_hist) and torch.equal(a.Dn, b.Dn)


@pytest.mark.parametrize("variant,chunk", [("yuma3", 0), ("yuma4", 5), ("yuma1", 0), ("yuma2", 4)])
def test_graph_replay_equals_direct_run(variant, chunk):
    """yuma_graph_create captures a whole multi-epoch run into one HIP graph;
    every replay must equal a direct yuma_run bitwise, including after the
    inputs are refilled in place, and the graph holds only device work
    (no host nodes): one kernel per phase per chunk."""
    E, N, V, M = 12, 2, 64, 512
    W = torch.from_numpy(synth.weights(0x6A, E, N, V, M)).cuda()
    S = torch.from_numpy(synth.stakes(0x6A, E, N, V, period=3)).cuda()
    vid = VARIANT_ID[variant]
    cfg = config_from({"liquid_alpha": True} if variant == "yuma4" else {})
    prm = [engine.make_params(vid, cfg)] * N
    g = engine.RunGraph(vid, prm, W, S, want_hist=True, chunk_epochs=chunk)
    assert g.nodes() >= 7
    for seed in (0x6A, 0x6B):
        W.copy_(torch.from_numpy(synth.weights(seed, E, N, V, M)))
        S.copy_(torch.from_numpy(synth.stakes(seed, E, N, V, period=3)))
        r = g.launch()
        ref = engine.run(vid, prm, W, S, want_hist=True, chunk_epochs=chunk)
        torch.cuda.synchronize()
        for a, b in ((r.Dn, ref.Dn), (r.C, ref.C), (r.I, ref.I), (r.B_hist, ref.B_hist),
                     (r.B_final, ref.B_final)):
            assert torch.equal(a, b)
    g.close()


@pytest.mark.parametrize("V,M,kind", [(256, 4096, "synth"), (64, 300, "randw"), (200, 130, "randw"),
                                      (33, 65, "synth"), (256, 1024, "nan_inf")])
def test_consensus_histogram_finish_equals_bisection(V, M, kind):
    """The exact-stake histogram finish of the consensus search (default) and
    the plain bisection (yuma_params_t.flags YUMA_FLAG_NO_HIST) give
    bitwise-equal consensus on inputs
    whose stakes are multiples of 2^-24 (synth.stakes sums to 2^20), across
    kappa / precision settings and bracket widths above the 64-bin limit
    (random-float weights); and both match the oracle. The nan_inf kind puts
    NaN / +inf / -inf / negative weights into some columns."""
    E = 3
    S = synth.stakes(0x5EEDC0 + V, E, 1, V, period=2)
    if kind == "synth":
        W = synth.weights(0x5EEDC0 + M, E, 1, V, M)
    else:
        rng = np.random.default_rng(V * 7 + M)
        W = rng.random((E, 1, V, M), dtype=np.float32)
        W[:, :, :, 0] = 0.0
        if kind == "nan_inf":
            W[0, 0, 3, 5] = np.nan
            W[1, 0, 7, 9] = np.inf
            W[1, 0, 8, 11] = -np.inf
            W[2, 0, 1, 13] = -0.5
    for spec in ({}, {"kappa": 0.3}, {"kappa": 0.7}, {"consensus_precision": 1000}, {"consensus_precision": 10000000}):
        cfg = config_from(spec)
        vid = engine.VARIANT_YUMA3
        prm = [engine.make_params(vid, cfg)]
        nohist = [engine.make_params(vid, cfg)]
        nohist[0].flags = engine.FLAG_NO_HIST
        Wt, St = torch.from_numpy(W), torch.from_numpy(S)
        tag = f"{kind} {V}x{M} {spec}"
        bits = lambda t: t.contiguous().view(torch.int32)  # NaN-safe bitwise compare
        a = engine.run(vid, prm, Wt, St, want_hist=True)
        b = engine.run(vid, nohist, Wt, St, want_hist=True)
        torch.cuda.synchronize()
        assert torch.equal(a.C, b.C), tag
        assert torch.equal(bits(a.B_hist), bits(b.B_hist)) and torch.equal(bits(a.Dn), bits(b.Dn)), tag
        if kind != "nan_inf":
            ref = orc.run("Yuma 3 (Rhef)", W[:, 0], S[:, 0], cfg)
            np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"], err_msg=tag)
