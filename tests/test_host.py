"""Host-side logic and the C-ABI library surface (CPU only, no compute calls)."""

import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT
from yuma_simulation._internal import cases as C
from yuma_simulation._internal import engine, wide, synth
from yuma_simulation._internal import yumas as Y
from yuma_simulation._internal.simulation_utils import VERSION_TABLE, resolve_version


def header_functions():
    text = open(os.path.join(ROOT, "include", "yuma_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(yuma_[a-z_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = engine.load_library()
    names = header_functions()
    assert set(names) == set(engine.EXPORTED_SYMBOLS), names
    for name in names:
        assert hasattr(lib, name), name
    assert engine.version().startswith("yuma_hip")


def test_params_struct_layout_matches_header():
    # the header promises 128 bytes; offsets of the double block are 8-aligned
    assert ctypes.sizeof(engine.YumaParamsC) == 128
    assert engine.YumaParamsC.ln_num.offset == 80
    assert ctypes.sizeof(engine.YumaOutputsC) == 8 * len(engine.OUTPUT_FIELDS)


def test_workspace_bytes_monotone():
    a = engine.workspace_bytes(3, 1, 10, 256, 4096, False)
    b = engine.workspace_bytes(3, 1, 20, 256, 4096, False)
    c = engine.workspace_bytes(3, 1, 10, 256, 4096, True)
    assert 0 < a < b and a < c


def test_compute_without_gpu_fails_loudly():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(engine.EngineUnavailable):
        Y.Yuma(torch.rand(4, 8), torch.rand(4))


def test_engine_limits_raise_clear_errors():
    """the engine's limits (consensus_precision <= 2**30,
    V <= 2**20 validators; the reference has neither) surface as EngineError
    with the limit named, before any GPU work (DESIGN.md §3 'Limits'). Above
    1024 validators the engine streams each miner column (round 5): such a
    subnet is no longer refused."""
    big = 2**20 + 1
    with pytest.raises(engine.EngineError, match=str(2**20)):
        engine.run(engine.VARIANT_YUMA4, [], torch.zeros(1, 1, big, 1), torch.zeros(1, 1, big))
    engine.check_limits(1025, 8)  # within the limits now
    engine.check_limits(2**20, 8)
    cfg = Y.YumaConfig(simulation=Y.SimulationHyperparameters(consensus_precision=2**31))
    with pytest.raises(engine.EngineError, match="2\\*\\*30"):
        Y.Yuma(torch.rand(4, 8), torch.rand(4), config=cfg)
    assert engine.make_params(engine.VARIANT_YUMA1, Y.YumaConfig(
        simulation=Y.SimulationHyperparameters(consensus_precision=2**30))).bisect_iters == 30


def test_config_defaults_and_flattening():
    cfg = Y.YumaConfig()
    assert (cfg.kappa, cfg.bond_penalty, cfg.total_epoch_emission) == (0.5, 1.0, 100.0)
    assert (cfg.validator_emission_ratio, cfg.total_subnet_stake, cfg.consensus_precision) == (0.41, 1e6, 100_000)
    assert (cfg.bond_alpha, cfg.liquid_alpha, cfg.alpha_high, cfg.alpha_low) == (0.1, False, 0.9, 0.7)
    assert (cfg.decay_rate, cfg.capacity_alpha) == (0.1, 0.1)
    assert cfg.override_consensus_high is None and cfg.override_consensus_low is None
    cfg2 = Y.YumaConfig(simulation=Y.SimulationHyperparameters(kappa=0.7), yuma_params=Y.YumaParams(bond_alpha=0.3))
    assert cfg2.kappa == 0.7 and cfg2.bond_alpha == 0.3


def test_names_and_dispatch():
    n = Y.YumaSimulationNames()
    assert n.YUMA_RUST == "Yuma 0 (subtensor)" and n.YUMA4_LIQUID.endswith("liquid alpha on")
    assert len(VERSION_TABLE) == 9
    assert resolve_version(n.YUMA31) == (engine.VARIANT_YUMA3, engine.RESET_ALWAYS)
    assert resolve_version(n.YUMA4) == (engine.VARIANT_YUMA4, engine.RESET_IF_ZERO_CONSENSUS)
    with pytest.raises(ValueError, match="Invalid Yuma function."):
        resolve_version("Yuma 5")


def test_bisection_trip_count():
    assert engine.bisect_iterations(100_000) == 17
    assert engine.bisect_iterations(1000) == 10
    assert engine.bisect_iterations(1) == 0
    with pytest.raises(ZeroDivisionError):
        engine.bisect_iterations(0)


def test_param_rounding_follows_python_then_fp32():
    cfg = Y.YumaConfig(simulation=Y.SimulationHyperparameters(kappa=0.3, bond_penalty=0.99),
                       yuma_params=Y.YumaParams(bond_alpha=0.025, decay_rate=0.1))
    p = engine.make_params(engine.VARIANT_YUMA4, cfg)
    assert p.kappa == float(np.float32(0.3))
    assert p.one_minus_bond_penalty == float(np.float32(1 - 0.99))
    assert p.one_minus_bond_alpha == float(np.float32(1 - 0.025))
    assert p.decay_keep == float(np.float32(0.9))
    assert p.maxint == 2.0**64
    assert p.liquid_mode == engine.LIQUID_OFF


def test_liquid_override_modes():
    mk = lambda **kw: engine.make_params(engine.VARIANT_YUMA1, Y.YumaConfig(yuma_params=Y.YumaParams(liquid_alpha=True, **kw)))
    assert mk().liquid_mode == engine.LIQUID_QUANTILE and mk().override_flags == 0
    p = mk(override_consensus_high=0.5)
    assert p.override_flags == engine.OVR_HIGH
    p = mk(override_consensus_high=0.5, override_consensus_low=0.5)
    assert p.liquid_mode == engine.LIQUID_QUANTILE and p.override_flags & engine.OVR_FORCE_Q99
    p = mk(override_consensus_high=0.5, override_consensus_low=0.1)
    assert p.liquid_mode == engine.LIQUID_CONST_AB
    a = (np.log(1 / 0.9 - 1) - np.log(1 / 0.7 - 1)) / (0.1 - 0.5)
    assert p.const_a == float(np.float32(a))
    # Yuma3 ignores liquid alpha entirely (reference yumas.py:399-491)
    p3 = engine.make_params(engine.VARIANT_YUMA3, Y.YumaConfig(yuma_params=Y.YumaParams(liquid_alpha=True, alpha_high=1.0)))
    assert p3.liquid_mode == engine.LIQUID_OFF
    with pytest.raises(ValueError):  # math.log(0), as the reference raises
        mk(alpha_high=1.0)


def test_reset_without_metadata_never_fires():
    p = engine.make_params(engine.VARIANT_YUMA3, Y.YumaConfig(), reset_mode=engine.RESET_ALWAYS)
    assert p.reset_mode == engine.RESET_NONE


def test_reset_index_follows_python_indexing():
    """run_simulation indexes B_state[:, idx] / scw[idx] (simulation_utils.py:63-85)."""
    mk = lambda mode, e, i, M=12, E=8: engine.make_params(
        engine.VARIANT_YUMA3, Y.YumaConfig(), reset_mode=mode, reset_epoch=e, reset_index=i, n_miners=M, n_epochs=E)
    p = mk(engine.RESET_ALWAYS, 3, -3)
    assert (p.reset_mode, p.reset_epoch, p.reset_index, p.flags) == (engine.RESET_ALWAYS, 3, 9, 0)
    p = mk(engine.RESET_IF_ZERO_CONSENSUS, 3, -12)
    assert p.reset_index == 0
    # None: B_state[:, None] = 0.0 zeroes every column (Yuma 3.1) ...
    p = mk(engine.RESET_ALWAYS, 3, None)
    assert p.reset_mode == engine.RESET_ALWAYS and p.flags & engine.FLAG_RESET_ALL_COLUMNS
    # ... while scw[None] == 0.0 has no truth value for M > 1 (Yuma 3.2 / 4)
    with pytest.raises(RuntimeError):
        mk(engine.RESET_IF_ZERO_CONSENSUS, 3, None)
    p = mk(engine.RESET_IF_ZERO_CONSENSUS, 3, None, M=1)
    assert p.reset_mode == engine.RESET_IF_ZERO_CONSENSUS and p.reset_index == 0 and p.flags == 0
    for bad in (12, -13):
        with pytest.raises(IndexError):
            mk(engine.RESET_ALWAYS, 3, bad)
    # the statement is never reached at epoch 0 (B_state is None) or past the run
    for e in (0, 8, -1):
        assert mk(engine.RESET_ALWAYS, e, 99).reset_mode == engine.RESET_NONE
        assert mk(engine.RESET_IF_ZERO_CONSENSUS, e, None).reset_mode == engine.RESET_NONE
    assert mk(engine.RESET_ALWAYS, None, 99).reset_mode == engine.RESET_NONE
    with pytest.raises(ValueError):  # a negative index cannot be resolved without M
        engine.make_params(engine.VARIANT_YUMA3, Y.YumaConfig(), reset_mode=engine.RESET_ALWAYS,
                           reset_epoch=3, reset_index=-1)


def test_reset_packing_equals_reference_statement():
    """the packed reset against the reference's own statements run
    in torch (simulation_utils.py:63-64 Yuma 3.1, :68-74 / :79-85 Yuma 3.2 / 4
    with scw all zero so the condition holds wherever it is defined): for
    every epoch of the run, which columns are zeroed, or the error raised.
    Covers float / bool / numpy epochs, 0-d and one-element tensors / arrays
    (truthy like their element), tensors / arrays of other sizes
    (no truth value: the reference raises) and bool / numpy indices."""
    M, E = 5, 6

    def reference(mode, e_ref, idx):
        out = {}
        for epoch in range(1, E):  # B_state exists from epoch 1 on
            try:
                if not epoch == e_ref:
                    continue
            except (RuntimeError, ValueError):  # a tensor / array without a truth value
                return "raise"
            B = torch.ones(2, M)
            if mode == engine.RESET_IF_ZERO_CONSENSUS:
                try:
                    fire = bool(torch.zeros(M)[idx] == 0.0)
                except RuntimeError:
                    return "raise"
                if not fire:
                    continue
            B[:, idx] = 0.0
            cols = frozenset(int(c) for c in (B[0] == 0).nonzero().flatten())
            if cols:
                out[epoch] = cols
        return out

    def packed(mode, e_ref, idx):
        try:
            p = engine.make_params(engine.VARIANT_YUMA3, Y.YumaConfig(), reset_mode=mode, reset_epoch=e_ref,
                                   reset_index=idx, n_miners=M, n_epochs=E)
        except (RuntimeError, ValueError):
            return "raise"
        if p.reset_mode == engine.RESET_NONE:
            return {}
        cols = range(M) if p.flags & engine.FLAG_RESET_ALL_COLUMNS else [p.reset_index]
        return {p.reset_epoch: frozenset(cols)}

    epochs = [3, 3.0, 3.5, True, False, np.int64(2), 0, -1, 6, "3", None,
              torch.tensor(3), torch.tensor([3]), torch.tensor(3.0), torch.tensor(3.5), torch.tensor(True),
              np.array(2), np.array([4.0]), torch.tensor([3, 4]), np.array([3, 4]), torch.tensor([]), np.array([])]
    indices = [2, -1, np.int64(4), True, False, None]
    for mode in (engine.RESET_ALWAYS, engine.RESET_IF_ZERO_CONSENSUS):
        for e_ref in epochs:
            for idx in indices:
                assert packed(mode, e_ref, idx) == reference(mode, e_ref, idx), (mode, e_ref, idx)


def test_shard_params_keeps_all_columns_reset():
    p = engine.make_params(engine.VARIANT_YUMA3, Y.YumaConfig(), reset_mode=engine.RESET_ALWAYS,
                           reset_epoch=3, reset_index=None, n_miners=300, n_epochs=8)
    out = [wide.shard_params([p], c)[0] for c in wide.column_ranges(300, 3)]
    assert all(q.reset_mode == engine.RESET_ALWAYS and q.flags & engine.FLAG_RESET_ALL_COLUMNS for q in out)


def test_cases_surface():
    assert len(C.cases) == 14 and list(C.class_registry) == [f"Case {i}" for i in range(1, 15)]
    c1 = C.create_case("Case 1")
    W = c1.weights_epochs
    assert len(W) == 40 and W[1].tolist() == [[0.0, 1.0], [1.0, 0.0], [1.0, 0.0]]
    assert c1.stakes_epochs[0].tolist() == pytest.approx([0.8, 0.1, 0.1])
    c9 = C.create_case("Case 9")
    assert c9.stakes_epochs[6].tolist() == pytest.approx([0.8, 0.2, 0.0])
    assert C.create_case("Case 5").reset_bonds_epoch == 20
    with pytest.raises(ValueError):
        C.create_case("Case 99")
    with pytest.raises(ValueError):
        C.Case1(base_validator="nobody")
    assert C.create_case("Case 1", num_epochs=7).packed_weights().shape == (7, 3, 2)
    # the returned lists are copies: mutating one does not leak into the next access
    W[0][0, 0] = 42.0
    assert c1.weights_epochs[0][0, 0] == 1.0


def test_synth_exactness_properties():
    W = synth.weights(5, 2, 2, 64, 4096)
    assert W.dtype == np.float32 and np.all(W == np.floor(W))
    rs = W.astype(np.float64).sum(axis=-1)
    assert rs.max() < 2**24 and rs.min() >= 32
    S = synth.stakes(5, 3, 2, 64, period=2)
    assert np.all(S.astype(np.int64).sum(axis=-1) == 2**20)
    assert np.array_equal(S[0], S[1]) and not np.array_equal(S[1], S[2])
    # deterministic and scenario-distinct
    assert np.array_equal(W, synth.weights(5, 2, 2, 64, 4096))
    assert not np.array_equal(W[:, 0], W[:, 1])


def test_sheet_versions_match_reference_scripts():
    """sheet_yuma_versions() is the list both reference scripts sweep
    (scripts/total_dividends_sheet_generator.py:25-48), as captured in specs."""
    from dataclasses import asdict

    from golden import specs
    from yuma_simulation._internal.simulation_utils import SHEET_BOND_PENALTIES, sheet_yuma_versions
    from yuma_simulation._internal.yumas import YumaParams

    got = sheet_yuma_versions()
    assert [v for v, _ in got] == specs.VERSIONS
    assert list(SHEET_BOND_PENALTIES) == specs.BETAS
    for (_, params), over in zip(got, specs.SHEET_PARAMS):
        assert asdict(params) == asdict(YumaParams(**over))


def test_scripts_import_without_gpu():
    import importlib
    import os
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    for name in ("scripts.total_dividends_sheet_generator", "scripts.charts_table_generator"):
        assert callable(importlib.import_module(name).main)


def test_bench_line_helpers(monkeypatch):
    """bench.py's phase -> kernel names and committed PMC traffic lookup (the
    pieces of the JSON line that need no GPU). The lookup is checked as if
    this library were the build the committed records were measured on
    (bench pairs a record only with its own build: test below)."""
    import json
    import sys

    sys.path.insert(0, ROOT)
    import bench

    recs = json.load(open(bench.TRAFFIC_JSON))
    ids = {r.get("build_id") for r in recs}
    assert len(ids) == 1, f"the committed PMC records come from several builds: {ids}"
    monkeypatch.setattr(bench, "engine_build_id", lambda: next(iter(ids)))

    for variant in range(5):
        for phase in engine.PHASES:
            assert bench.kernel_of(phase, variant).startswith("k_")
    assert bench.kernel_of("bonds", engine.VARIANT_YUMA3) == "k_bonds_elem"
    assert bench.kernel_of("bonds", engine.VARIANT_YUMA4, shared=True, N=512) == "k_bonds_grp"
    assert bench.kernel_of("bonds", engine.VARIANT_YUMA1) == "k_bonds_elem"  # rank-formed column sums
    assert bench.kernel_of("bonds", engine.VARIANT_YUMA2) == "k_bonds_elem"
    assert bench.kernel_of("bonds", engine.VARIANT_RUST) == "k_bonds_cn"
    assert bench.kernel_of("bonds", engine.VARIANT_YUMA1, V=64) == "k_bonds"  # below 65 validators
    assert bench.kernel_of("rank", engine.VARIANT_YUMA3) == "k_rank_s"
    assert bench.kernel_of("rank", engine.VARIANT_YUMA2) == "k_rank_sw"  # + bond column sums
    assert bench.kernel_of("rank", engine.VARIANT_YUMA3, M=65536) == "k_rank_sw"
    assert bench.kernel_of("consensus", engine.VARIANT_YUMA3) == "k_consensus_p"
    assert bench.kernel_of("consensus", engine.VARIANT_YUMA4, shared=True, N=512) == "k_consensus_w"
    assert bench.kernel_of("consensus", engine.VARIANT_YUMA3, V=64) == "k_consensus_w"
    key = {"V": 256, "M": 4096, "epochs": 1000, "scenarios_per_gpu": 1, "version": "Yuma 3 (Rhef)",
           "bond_history": True}
    pmc = bench.load_traffic(key)
    assert pmc is not None and pmc["k_bonds_elem"] > 8e6
    # every bench config has a committed traffic record (c3: the grouped scan)
    c3 = bench.load_traffic({"V": 256, "M": 4096, "epochs": 32, "scenarios_per_gpu": 512,
                             "version": "Yuma 4 (Rhef+relative bonds)", "bond_history": False})
    assert c3 is not None and "k_bonds_grp" in c3
    c4 = bench.load_traffic({"V": 256, "M": 65536, "epochs": 100, "scenarios_per_gpu": 1,
                             "version": "Yuma 3 (Rhef)", "bond_history": False})
    assert c4 is not None and "k_consensus_p" in c4 and "k_rank_sw" in c4  # round-5 kernels
    assert bench.load_traffic(dict(key, M=1)) is None
    assert bench.contract_bytes(256, 4096, 3) == 12_617_728


def test_bench_consensus_classes():
    """The c3 line's consensus-class count (what k_classes shares on the GPU:
    equal kappa bits, bisection trip count and histogram switch): 16 kappa
    values per GPU share of the 4096-point grid."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    params = [engine.make_params(engine.VARIANT_YUMA4, bench.sweep_config(g)) for g in range(512)]
    assert bench.consensus_classes(params) == 16
    params[3].flags |= engine.FLAG_NO_HIST  # the histogram switch splits a class
    assert bench.consensus_classes(params) == 17


def test_bench_input_seed_per_config():
    """an N-rank c3 line sweeps ONE subnet trajectory (every rank
    the same inputs, its own share of the grid); c2 replicas are independent
    subnets, one seed per rank."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    assert {bench.input_seed("c3", 0x5EED0003, r) for r in range(8)} == {0x5EED0003}
    assert len({bench.input_seed("c2", 0x5EED0002, r) for r in range(8)}) == 8
    assert bench.input_seed("c2", 0x5EED0002, 0) == 0x5EED0002


def _grp_omba(ba_param: float, omba_param: float) -> np.float32:
    """k_bonds_grp's operand for a fixed-alpha scenario (p_corr):
    (1 - bond_alpha) + corr, corr = one_minus_bond_alpha - (1 - bond_alpha),
    a NaN corr (bond_alpha = +-inf) replaced by 0, all in fp32."""
    one = np.float32(1.0)
    ba, omba = np.float32(ba_param), np.float32(omba_param)
    with np.errstate(invalid="ignore", over="ignore"):
        x = one - ba
        corr = omba - x
        if corr != corr:
            corr = np.float32(0.0)
        return x + corr


def test_grp_one_minus_alpha_correction():
    """The sweep scan rebuilds one_minus_bond_alpha = f32(1 - bond_alpha)
    (double, engine.make_params) from f32(bond_alpha) bit for bit, for every
    bond_alpha a YumaConfig can carry (yumas.py:566-575 uses 1 - bond_alpha)."""
    rng = np.random.default_rng(7)
    alphas = list(rng.random(200_000)) + list(rng.random(20_000) * 1e-6) + list(1 - rng.random(20_000) * 1e-6)
    alphas += list(10.0 ** rng.uniform(-45, 40, 20_000)) + list(-(10.0 ** rng.uniform(-45, 40, 5_000)))
    alphas += [0.0, -0.0, 1.0, 0.5, 0.1, 0.9, 0.025, 1e-9, 1 - 1e-9, 1 - 2**-24, 1 - 2**-25, 1 + 2**-23,
               2**-126, 2**-149, 3.4e38, 1e39, -1e39, float("inf"), float("-inf")]
    from bench import SWEEP_BOND_ALPHA  # the c3 grid's bond_alpha values
    alphas += list(SWEEP_BOND_ALPHA)
    bad = []
    for a in alphas:
        cfg = Y.YumaConfig(yuma_params=Y.YumaParams(bond_alpha=float(a)))
        p = engine.make_params(engine.VARIANT_YUMA4, cfg)
        got = _grp_omba(p.bond_alpha, p.one_minus_bond_alpha)
        want = np.float32(p.one_minus_bond_alpha)
        if got.view(np.uint32) != want.view(np.uint32):
            bad.append((a, float(got), float(want)))
    assert not bad, bad[:5]


def test_library_build_id_is_this_source():
    """yuma_build_id stamps the SHA-256 prefix of the engine source + header
    the library was compiled from: the in-tree library is this tree's source
    (bench.py pairs committed counter records with runs by this id)."""
    import __graft_entry__ as g
    from yuma_simulation._internal import engine

    assert engine.build_id() == g.source_build_id()


def test_bench_ignores_counter_records_of_another_build(tmp_path, monkeypatch):
    """a PMC / SQ record measured on another library build
    is never paired with this run's timings."""
    import json

    import bench

    key = {"V": 256, "M": 4096, "epochs": 1000, "scenarios_per_gpu": 1, "version": "Yuma 3 (Rhef)",
           "bond_history": True}
    rec = {"workload": key, "build_id": "src-0000000000000000",
           "kernels": {"k_bonds_elem": {"hbm_bytes_per_scenario_epoch": 1.0}}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps([rec]))
    monkeypatch.setattr(bench, "TRAFFIC_JSON", str(p))
    monkeypatch.setattr(bench, "engine_build_id", lambda: "src-1111111111111111")
    assert bench.load_traffic(key) is None
    monkeypatch.setattr(bench, "engine_build_id", lambda: "src-0000000000000000")
    assert bench.load_traffic(key) == {"k_bonds_elem": 1.0}


def test_committed_counter_records_are_this_build():
    """Every committed PMC / SQ record that bench.py pairs with its timings was
    measured on the library this tree builds: an engine
    change without a fresh profiling pass fails here instead of pairing stale
    counters with new kernels (bench.py would print null for them)."""
    import json
    import sys

    import __graft_entry__ as g

    sys.path.insert(0, ROOT)
    import bench

    bid = g.source_build_id()
    for path in (bench.TRAFFIC_JSON, bench.SQ_JSON):
        recs = json.load(open(path))
        assert recs, path
        for r in recs:
            assert r.get("build_id") == bid, f"{os.path.relpath(path, ROOT)} {r['workload']}: {r.get('build_id')} != {bid}"


def test_group_dividend_ratio_equals_per_run():
    """run_simulations forms the dividend ratio of a whole batch in one pass of
    the same elementwise ops (simulation_utils.py:95-107 restated): bitwise
    the per-run results, on random stakes / dividends with zero stakes."""
    import torch

    from yuma_simulation._internal import simulation_utils as su
    from yuma_simulation._internal.yumas import YumaConfig

    g = torch.Generator().manual_seed(5)
    S = torch.rand(40, 7, 3, generator=g)
    S[3, 2, 1] = 0.0
    Dn = torch.rand(40, 7, 3, generator=g)
    cfg = YumaConfig()
    whole = su._dividend_ratio(cfg, S, Dn)
    for j in range(7):
        one = su._dividend_ratio(cfg, S[:, j].contiguous(), Dn[:, j].contiguous())
        assert np.array_equal(whole[:, j], one)


def test_make_params_cache_matches_and_separates():
    from yuma_simulation._internal.yumas import SimulationHyperparameters, YumaConfig, YumaParams

    a = YumaConfig(yuma_params=YumaParams(bond_alpha=0.2))
    b = YumaConfig(yuma_params=YumaParams(bond_alpha=0.2))
    c = YumaConfig(simulation=SimulationHyperparameters(kappa=-0.0))
    d = YumaConfig(simulation=SimulationHyperparameters(kappa=0.0))
    pa = engine.make_params_cached(engine.VARIANT_YUMA4, a)
    assert engine.make_params_cached(engine.VARIANT_YUMA4, b) is pa
    assert bytes(pa) == bytes(engine.make_params(engine.VARIANT_YUMA4, a))
    assert engine.make_params_cached(engine.VARIANT_YUMA3, a) is not pa
    pc, pd = engine.make_params_cached(3, c), engine.make_params_cached(3, d)
    assert pc is not pd and bytes(pc) == bytes(engine.make_params(3, c))


def test_prefix_totals_equal_list_sums():
    """The sheet's totals path (simulation_utils._prefix_total over numpy's
    sequential running sums) gives the bits of summing the per-epoch lists
    with Python's sum() (charts_utils.py:19 restated): prefixes shorter, equal
    and longer than the run, an empty and a negative slice, -0.0 terms."""
    from yuma_simulation._internal import simulation_utils as su

    rng = np.random.default_rng(11)
    E = 40
    x = rng.random((E, 3)) * 10.0 ** rng.integers(-8, 8, (E, 3))
    x[:, 2] = -0.0
    x[5, 1] = 0.0
    cs = np.cumsum(x, axis=0)
    cols = x.T.tolist()
    for n in (0, 1, 7, 39, 40, 55, -3):
        got = su._prefix_total(cs, E, n)
        want = [sum(c[:n]) for c in cols]
        assert [type(g) for g in got] == [type(w) for w in want], n
        assert [repr(g) for g in got] == [repr(w) for w in want], n


def test_sheet_frame_block_equals_row_frame(capsys):
    """_sheet_frame_totals' float64 block equals the row-dict frame (same
    columns, dtypes, CSV text and zero-base warnings) on the reference's
    cases, and keeps the row form for int totals (an empty epoch range)."""
    from yuma_simulation._internal import simulation_utils as su

    vers = su.sheet_yuma_versions()
    rng = np.random.default_rng(3)
    for zero in (False, True):
        tots = []
        for case in C.cases:
            for _ in vers:
                t = {v: float(rng.random()) for v in case.validators}
                if zero:
                    t[case.base_validator] = 0.0
                tots.append(t)
        lists = [[t[v] for v in C.cases[i // len(vers)].validators] for i, t in enumerate(tots)]
        a = su._sheet_frame_totals(C.cases, vers, lists)
        wa = capsys.readouterr().out
        rows = []
        it = iter(tots)
        for case in C.cases:
            row = {"Case": case.name}
            std_of = dict(zip(case.validators, su._STANDARDIZED))
            for version, _ in vers:
                t = next(it)
                if t.get(case.base_validator) in (None, 0.0):
                    print(f"Warning: Base validator '{case.base_validator}' has zero or missing total dividends.")
                by_std = {std_of[v]: t.get(v, 0.0) for v in case.validators}
                for std in su._STANDARDIZED:
                    row[f"{std} - {version}"] = by_std.get(std, 0.0)
            rows.append(row)
        b = pd_frame(rows)
        wb = capsys.readouterr().out
        assert list(a.columns) == list(b.columns) and a.dtypes.equals(b.dtypes)
        assert a.to_csv(index=False, float_format="%.6f") == b.to_csv(index=False, float_format="%.6f")
        assert a.to_csv(index=False) == b.to_csv(index=False)
        assert wa == wb and (zero == (len(wa) > 0))
    ints = [[0 for v in case.validators] for case in C.cases for _ in vers]
    c = su._sheet_frame_totals(C.cases, vers, ints)
    capsys.readouterr()
    assert str(c.dtypes.iloc[1]) == "int64"


def pd_frame(rows):
    import pandas as pd

    return pd.DataFrame(rows)
