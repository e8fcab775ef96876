"""Pin the CPU oracle (oracle/yuma_oracle.py) against golden vectors captured
from the reference (tests/golden/make_golden.py). CPU only."""

import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_close
from golden import specs
from oracle import yuma_oracle as orc
from yuma_simulation._internal import synth
from yuma_simulation._internal.cases import cases
from yuma_simulation._internal.yumas import SimulationHyperparameters, YumaConfig, YumaParams


def config_from(spec: dict) -> YumaConfig:
    sim, par = specs.split_spec(spec)
    return YumaConfig(simulation=SimulationHyperparameters(**sim), yuma_params=YumaParams(**par))


def sheet_config(beta, vi):
    return YumaConfig(simulation=SimulationHyperparameters(bond_penalty=beta),
                      yuma_params=YumaParams(**specs.SHEET_PARAMS[vi]))


@pytest.fixture(scope="module")
def sheet(golden):
    with open(os.path.join(GOLDEN, "sheet.json")) as f:
        meta = json.load(f)
    return golden("sheet.npz"), meta


@pytest.mark.parametrize("bi", range(4))
def test_oracle_sheet_runs(sheet, bi):
    """All 14 cases x 9 versions at one bond_penalty: per-epoch consensus
    (exact), dividends, bonds, incentives."""
    g, meta = sheet
    beta = specs.BETAS[bi]
    assert meta["versions"] == specs.VERSIONS
    for ci, case in enumerate(cases):
        assert case.name == meta["cases"][ci]
        assert case.validators == meta["validators"][ci]
        W = case.packed_weights().numpy()
        S = case.packed_stakes().numpy()
        for vi, version in enumerate(specs.VERSIONS):
            cfg = sheet_config(beta, vi)
            out = orc.run(version, W, S, cfg, case.reset_bonds_epoch, case.reset_bonds_index,
                          validators=case.validators)
            tag = f"b{beta} {case.name[:7]} {version}"
            np.testing.assert_array_equal(out["C"], g["consensus"][bi, ci, vi], err_msg=tag)
            div = np.array([out["dividends"][v] for v in case.validators]).T
            assert_close(div, g["dividends"][bi, ci, vi], what=tag + " dividends")
            assert_close(out["B"], g["bonds"][bi, ci, vi], what=tag + " bonds")
            assert_close(out["I"], g["incentives"][bi, ci, vi], what=tag + " incentives")
            assert_close(out["Dn"], g["dn"][bi, ci, vi], what=tag + " Dn")


def test_oracle_sheet_csv_anchor(sheet):
    """Known-answer anchors quoted in SURVEY §8c (beta=1.0, Case 1)."""
    g, _ = sheet
    bi, ci = 3, 0
    want = {  # version index -> validators A/B/C total dividends
        0: (1.745287, 1.241205, 1.196481), 1: (1.680764, 1.527371, 1.426488),
        3: (1.639736, 1.486438, 1.385649), 4: (1.676663, 1.540661, 1.446037),
        7: (1.677617, 1.538392, 1.440640), 8: (1.690750, 1.504875, 1.368883),
    }
    for vi, tot in want.items():
        got = g["dividends"][bi, ci, vi].sum(axis=0)
        np.testing.assert_allclose(got, tot, atol=5e-7)


def _small_cases():
    for iname in ("synth16x64", "rand16x64", "edge3x5"):
        for variant in specs.VARIANTS:
            for cname in specs.CONFIGS:
                if cname.startswith("liquid") and variant == "yuma3":
                    continue
                yield iname, variant, cname


@pytest.mark.parametrize("iname,variant,cname", list(_small_cases()))
def test_oracle_epoch_small(golden, iname, variant, cname):
    g = golden("epoch_small.npz")
    cfg = config_from(specs.CONFIGS[cname])
    W0, S0 = g[f"in__{iname}__W0"], g[f"in__{iname}__S0"]
    W1, S1 = g[f"in__{iname}__W1"], g[f"in__{iname}__S1"]
    r0 = orc.epoch(variant, W0, S0, None, cfg)
    prev = r0["weight"] if variant == "yuma2" else None
    r1 = orc.epoch(variant, W1, S1, r0[orc.state_key(variant)].copy(), cfg, W_prev=prev)
    for step, r in (("e0", r0), ("e1", r1)):
        tag = f"out__{iname}__{variant}__{cname}__{step}"
        keys = [k[len(tag) + 2:] for k in g.files if k.startswith(tag + "__") and not k.endswith("__pyfloat")]
        assert set(keys) == set(r), f"{tag}: keys {sorted(set(keys) ^ set(r))}"
        for k in keys:
            exp = g[f"{tag}__{k}"]
            got = r[k]
            if f"{tag}__{k}__pyfloat" in g.files:
                assert isinstance(got, float), f"{tag} {k} should be a python float"
            if k == "server_consensus_weight":
                np.testing.assert_array_equal(got, exp, err_msg=f"{tag} {k}")
            else:
                assert_close(got, exp, what=f"{tag} {k}")


@pytest.mark.parametrize("sname", ["synth64x512", "rand32x256"])
def test_oracle_run_medium(golden, sname):
    g = golden("run_medium.npz")
    W, S = g[f"in__{sname}__W"], g[f"in__{sname}__S"]
    re, ri = (int(x) for x in g[f"in__{sname}__reset"])
    validators = [f"V{i}" for i in range(W.shape[1])]
    for vi, version in enumerate(specs.VERSIONS):
        cfg = sheet_config(0.5, vi)
        out = orc.run(version, W, S, cfg, re, ri, validators=validators)
        tag = f"out__{sname}__{vi}"
        np.testing.assert_array_equal(out["C"], g[f"{tag}__C"], err_msg=f"{tag} C")
        assert_close(out["Dn"], g[f"{tag}__Dn"], what=f"{tag} Dn")
        assert_close(out["I"], g[f"{tag}__I"], what=f"{tag} I")
        assert_close(out["B"][-1], g[f"{tag}__B_last"], what=f"{tag} B_last")
        assert_close(out["B"][0], g[f"{tag}__B_first"], what=f"{tag} B_first")
        div = np.array([out["dividends"][v] for v in validators]).T
        assert_close(div, g[f"{tag}__dividends"], what=f"{tag} dividends")


@pytest.fixture(scope="module")
def large_inputs(golden):
    g = golden("large.npz")
    W = synth.weights(specs.LARGE_SEED, 2, 1, 256, 4096)[:, 0]
    S = synth.stakes(specs.LARGE_SEED, 2, 1, 256)[:, 0]
    assert hashlib.sha256(np.ascontiguousarray(W).tobytes()).hexdigest()[:16] == str(g["in__W_sha"])
    np.testing.assert_array_equal(S, g["in__S"])
    return g, W, S


@pytest.mark.parametrize("name", list(specs.LARGE_SPECS))
def test_oracle_large(large_inputs, name):
    g, W, S = large_inputs
    variant = name.split("_")[0]
    cfg = config_from(specs.LARGE_SPECS[name])
    r0 = orc.epoch(variant, W[0], S[0], None, cfg)
    prev = r0["weight"] if variant == "yuma2" else None
    r1 = orc.epoch(variant, W[1], S[1], r0[orc.state_key(variant)].copy(), cfg, W_prev=prev)
    idx = g["sample_idx"]
    for step, r in (("e0", r0), ("e1", r1)):
        tag = f"out__{name}__{step}"
        np.testing.assert_array_equal(r["server_consensus_weight"], g[f"{tag}__server_consensus_weight"])
        for k in ("server_incentive", "server_rank", "server_prerank", "validator_reward",
                  "validator_reward_normalized"):
            assert_close(r[k], g[f"{tag}__{k}"], what=f"{tag} {k}")
        B = r[orc.state_key(variant)]
        assert_close(B.astype(np.float64).sum(axis=0), g[f"{tag}__B_colsum"], what=f"{tag} Bcol")
        assert_close(B.astype(np.float64).sum(axis=1), g[f"{tag}__B_rowsum"], what=f"{tag} Brow")
        assert_close(B[idx[:, 0], idx[:, 1]], g[f"{tag}__B_sample"], what=f"{tag} Bsample")
        if f"{tag}__bond_alpha" in g.files:
            assert_close(r["bond_alpha"], g[f"{tag}__bond_alpha"], what=f"{tag} bond_alpha")


def test_oracle_large_random_floats(golden):
    """Generic float inputs (not exactness-friendly): consensus decisions still
    match the reference on every column (SURVEY §0 fact 3 probe)."""
    g = golden("large.npz")
    Wr, Sr = synth.random_float_inputs(int(g["rand__W_seed"]), 1, 256, 4096)
    r = orc.epoch("yuma1", Wr[0], Sr[0], None, config_from({}))
    np.testing.assert_array_equal(r["server_consensus_weight"], g["rand__server_consensus_weight"])
    assert_close(r["server_incentive"], g["rand__server_incentive"])
    assert_close(r["validator_reward_normalized"], g["rand__validator_reward_normalized"])


def test_tie_columns_flags_exact_ties_only():
    """oracle.tie_columns (the summation-order tie window of yumas.py:203-204,
    :186, :211): a column whose stake sum above the bisection midpoint equals
    kappa exactly is flagged; on random inputs few columns are."""
    S = np.full(4, 0.25, np.float32)
    W = np.array([[2, 1, 0], [2, 1, 0], [0, 1, 2], [0, 1, 2]], np.float32)
    flags = orc.tie_columns(W, S, 0.5, 2**17)
    assert flags[0] and flags[2]  # stake 0.5 above every mid below 2/3: == kappa
    rng = np.random.default_rng(5)
    Wr = rng.random((16, 64), dtype=np.float32)
    Sr = rng.random(16, dtype=np.float32)
    assert 0 < (~orc.tie_columns(Wr, Sr, 0.5, 2**17)).sum() and orc.tie_columns(Wr, Sr, 0.5, 2**17).mean() < 0.2


# ---------------------------------------------------------------------------
# oracle/torch_cpu.py: the CPU baseline's restatement, bit-for-bit
# ---------------------------------------------------------------------------
def _torch_cases():
    for iname in ("synth16x64", "rand16x64", "edge3x5"):
        for variant in specs.VARIANTS:
            for cname in specs.CONFIGS:
                if cname.startswith("liquid") and variant == "yuma3":
                    continue
                yield iname, variant, cname


def _bits_equal(a, e, what):
    a = np.asarray(a.numpy() if hasattr(a, "numpy") else a)
    e = np.asarray(e)
    if a.dtype != e.dtype and a.dtype == np.float64 and e.dtype == np.float32:
        raise AssertionError(f"{what}: fp64 result where the reference has fp32")
    a = np.atleast_1d(a.astype(e.dtype))
    e = np.atleast_1d(e)
    assert a.shape == e.shape, what
    if e.dtype.kind == "f":
        u = np.uint32 if e.dtype.itemsize == 4 else np.uint64
        assert np.array_equal(a.view(u), e.view(u)) or np.array_equal(a, e, equal_nan=True), what
    else:
        assert np.array_equal(a, e), what


@pytest.mark.parametrize("iname,variant,cname", list(_torch_cases()))
def test_torch_cpu_structured_bit_identical_small(golden, iname, variant, cname):
    """The reference-structured torch restatement (SURVEY §8d baseline (i))
    reproduces the reference's full result dicts bit for bit."""
    import torch

    from oracle import torch_cpu as tc

    g = golden("epoch_small.npz")
    cfg = config_from(specs.CONFIGS[cname])
    B = prev = None
    for step in ("e0", "e1"):
        e = step[1]
        W = torch.from_numpy(g[f"in__{iname}__W{e}"])
        S = torch.from_numpy(g[f"in__{iname}__S{e}"])
        for mode in ("structured", "vectorised"):
            r = tc.epoch(variant, W, S, B, cfg, consensus=mode, W_prev=prev)
            tag = f"out__{iname}__{variant}__{cname}__{step}"
            keys = [k[len(tag) + 2:] for k in g.files if k.startswith(tag + "__") and not k.endswith("__pyfloat")]
            assert set(keys) == set(r), tag
            for k in keys:
                if f"{tag}__{k}__pyfloat" in g.files:
                    assert isinstance(r[k], float), f"{tag} {k} should be a python float"
                _bits_equal(r[k], g[f"{tag}__{k}"], f"{tag} {k} ({mode})")
        B = r[tc.state_key(variant)].clone()
        prev = r["weight"] if variant == "yuma2" else None


@pytest.mark.parametrize("name", ["yuma3", "yuma4", "yuma4_liquid"])
def test_torch_cpu_bit_identical_large(large_inputs, name):
    """256 x 4096 (the c2 shape), two epochs: consensus, rank, incentive,
    prerank, dividends and the sampled bonds bit-identical to the reference
    for both consensus forms (the benchmark's dyadic stakes make the
    vectorised column sums order-independent)."""
    import torch

    from oracle import torch_cpu as tc

    g, W, S = large_inputs
    variant = name.split("_")[0]
    cfg = config_from(specs.LARGE_SPECS[name])
    idx = g["sample_idx"]
    for mode in ("vectorised", "structured"):
        B = None
        for t, step in enumerate(("e0", "e1")):
            r = tc.epoch(variant, torch.from_numpy(W[t]), torch.from_numpy(S[t]), B, cfg, consensus=mode)
            B = r["validator_bonds"]
            tag = f"out__{name}__{step}"
            for k in ("server_consensus_weight", "server_incentive", "server_rank", "server_prerank",
                      "validator_reward", "validator_reward_normalized"):
                _bits_equal(r[k].numpy(), g[f"{tag}__{k}"], f"{tag} {k} ({mode})")
            Bn = B.numpy()
            _bits_equal(Bn[idx[:, 0], idx[:, 1]], g[f"{tag}__B_sample"], f"{tag} B_sample ({mode})")
            assert_close(Bn.astype(np.float64).sum(axis=0), g[f"{tag}__B_colsum"], rtol=1e-12, atol_frac=0,
                         what=f"{tag} B colsum ({mode})")


@pytest.mark.parametrize("bi", range(4))
def test_torch_cpu_run_simulation_matches_sheet(sheet, bi):
    """oracle/torch_cpu.run_simulation (the c5 CPU baseline) reproduces the
    reference's dividend lists of every sheet run bit for bit (the per-epoch
    Python floats the sheet CSVs are summed from)."""
    from oracle import torch_cpu as tc

    g, _ = sheet
    beta = specs.BETAS[bi]
    for ci, case in enumerate(cases):
        for vi, version in enumerate(specs.VERSIONS):
            div, bonds, inc = tc.run_simulation(version, case.weights_epochs, case.stakes_epochs,
                                                sheet_config(beta, vi), case.num_epochs, case.validators,
                                                case.reset_bonds_epoch, case.reset_bonds_index)
            got = np.array([div[v] for v in case.validators]).T
            tag = f"b{beta} {case.name[:7]} {version}"
            np.testing.assert_array_equal(got, g["dividends"][bi, ci, vi], err_msg=tag)


@pytest.mark.parametrize("bi", [0, 3])
def test_dividends_per_1000_tao_bitwise(sheet, bi):
    """The host-side dividend formatting of run_simulations
    (simulation_utils._dividends_per_1000_tao: the reference's tensor ops,
    then the Python-double ratio, simulation_utils.py:48-49,95-107) turns the
    reference's own normalised dividends into the reference's dividend lists
    bit for bit (CPU only: the golden Dn stand in for the engine's)."""
    import torch

    from yuma_simulation._internal.simulation_utils import _dividends_per_1000_tao

    g, _ = sheet
    beta = specs.BETAS[bi]
    for ci, case in enumerate(cases):
        W, S = case.packed_inputs()
        for vi in range(len(specs.VERSIONS)):
            cfg = sheet_config(beta, vi)
            Dn = torch.from_numpy(np.ascontiguousarray(g["dn"][bi, ci, vi]))
            div = _dividends_per_1000_tao(case, cfg, S, Dn)
            got = np.array([div[v] for v in case.validators]).T
            np.testing.assert_array_equal(got, g["dividends"][bi, ci, vi], err_msg=f"{case.name} {vi}")
            assert all(type(x) is float for v in case.validators for x in div[v])
