"""Wide subnet sharded by miner column.

CPU (not gpu): shard geometry, per-shard parameter records, and the
rank-ordered all-gather over gloo (world_size 2, uneven shard widths).
GPU: the five shard stages through the C-ABI, several shards in one process
and two processes (gloo) on one GPU, against the unsharded engine run — which
is itself pinned to the reference goldens and the oracle (test_gpu_parity.py)
— and directly against the oracle. Consensus levels, clip decisions and bond
states are bit-identical; dividends/incentives within 1e-5 relative (the
cross-shard sums associate differently than the one-GPU tile order)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import assert_close
from yuma_simulation._internal import engine, synth, wide
from yuma_simulation._internal.yumas import SimulationHyperparameters, YumaConfig, YumaParams


# ---------------------------------------------------------------------------
# host logic (no GPU)
# ---------------------------------------------------------------------------
def test_column_ranges_tile_aligned_and_cover():
    for M, k in [(64, 1), (300, 2), (300, 5), (65536, 8), (65536 + 7, 8), (4096, 3)]:
        rs = wide.column_ranges(M, k)
        assert len(rs) == k
        assert rs[0].start == 0 and rs[-1].stop == M
        for a, b in zip(rs, rs[1:]):
            assert a.stop == b.start and a.stop % wide.TILE == 0
        sizes = [len(r) for r in rs]
        assert max(sizes) - min(sizes) < 2 * wide.TILE
    with pytest.raises(ValueError):
        wide.column_ranges(100, 3)  # 2 tiles cannot make 3 shards


def test_shard_params_relocates_reset():
    cfg = YumaConfig()
    p = engine.make_params(engine.VARIANT_YUMA3, cfg, reset_mode=engine.RESET_ALWAYS,
                           reset_epoch=3, reset_index=130)
    cols = wide.column_ranges(300, 3)  # [0,128) [128,256) [256,300)
    out = [wide.shard_params([p], c)[0] for c in cols]
    assert [q.reset_mode for q in out] == [engine.RESET_NONE, engine.RESET_ALWAYS, engine.RESET_NONE]
    assert out[1].reset_index == 2 and out[1].reset_epoch == 3
    assert p.reset_index == 130  # the caller's record is untouched


def test_ordered_sum_is_shard_order():
    xs = [torch.tensor([1e8], dtype=torch.float32), torch.tensor([1.0]), torch.tensor([-1e8])]
    assert wide.ordered_sum(xs).item() == 0.0  # fp32, shard order: (1e8 + 1) - 1e8
    assert wide.ordered_sum([xs[0], xs[2], xs[1]]).item() == 1.0  # another order, another sum


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = wide.dist_gather()
        x = torch.arange(6 * (rank + 2), dtype=torch.float32).reshape(2, 3, rank + 2) + 100 * rank
        parts = g([x], [2, 3])
        same = g([torch.full((2, 2), float(rank))])
        assert [float(p[0, 0]) for p in same] == [0.0, 1.0]
        tot = wide.ordered_sum([torch.ones(4) * (r + 1) for r in range(world)])
        q.put((rank, [p.numpy() for p in parts], tot.numpy()))
    finally:
        dist.destroy_process_group()


def test_dist_gather_uneven_rank_order():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (parts, tot)) for r, parts, tot in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        parts, tot = got[r]
        assert [p.shape for p in parts] == [(2, 3, 2), (2, 3, 3)]
        for k in range(world):
            exp = np.arange(6 * (k + 2), dtype=np.float32).reshape(2, 3, k + 2) + 100 * k
            np.testing.assert_array_equal(parts[k], exp)
        np.testing.assert_array_equal(tot, np.full(4, 3.0, np.float32))


# ---------------------------------------------------------------------------
# GPU: shard stages through the C-ABI
# ---------------------------------------------------------------------------
E, V, M = 6, 40, 300


def _inputs(seed, N=2):
    W = synth.weights(seed, E, N, V, M)
    S = synth.stakes(seed, E, N, V, period=3)
    W[1, :, :, 150] = 0.0  # column 150 gets zero consensus at epoch 1 (reset-if-zero fires)
    return torch.from_numpy(W), torch.from_numpy(S)


CASES = {
    "rust": (engine.VARIANT_RUST, dict()),
    "rust_liquid": (engine.VARIANT_RUST, dict(liquid_alpha=True)),
    "yuma1": (engine.VARIANT_YUMA1, dict()),
    "yuma1_liquid": (engine.VARIANT_YUMA1, dict(liquid_alpha=True)),
    "yuma2": (engine.VARIANT_YUMA2, dict()),
    "yuma3": (engine.VARIANT_YUMA3, dict()),
    "yuma4_liquid": (engine.VARIANT_YUMA4, dict(liquid_alpha=True)),
}


def _params(variant, par, N, reset=None):
    out = []
    for j in range(N):
        cfg = YumaConfig(simulation=SimulationHyperparameters(kappa=0.45 + 0.1 * j),
                         yuma_params=YumaParams(**par))
        kw = {}
        if reset is not None:
            kw = dict(reset_mode=reset, reset_epoch=2, reset_index=150)
        out.append(engine.make_params(variant, cfg, **kw))
    return out


def _compare(sharded, ref, cols):
    C = torch.cat(sharded.C, dim=2).cpu().numpy()
    np.testing.assert_array_equal(C, ref.C.cpu().numpy())  # consensus: bit-identical
    Bf = torch.cat(sharded.B_final, dim=2).cpu().numpy()
    np.testing.assert_array_equal(Bf, ref.B_final.cpu().numpy())  # bond state: column-local
    Bh = torch.cat(sharded.B_hist, dim=3).cpu().numpy()
    np.testing.assert_array_equal(Bh, ref.B_hist.cpu().numpy())
    assert_close(torch.cat(sharded.I, dim=2).cpu().numpy(), ref.I.cpu().numpy(), what="I")
    assert_close(sharded.Dn.cpu().numpy(), ref.Dn.cpu().numpy(), what="Dn")


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("n_shards", [2, 3])
def test_wide_local_matches_unsharded(name, n_shards):
    variant, par = CASES[name]
    W, S = _inputs(0x5EED4 + n_shards)
    params = _params(variant, par, W.shape[1])
    ref = engine.run(variant, params, W, S, want_hist=True)
    got = wide.run_wide_local(variant, params, W, S, n_shards, want_hist=True)
    torch.cuda.synchronize()
    _compare(got, ref, wide.column_ranges(M, n_shards))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rust", "yuma2", "yuma3"])
@pytest.mark.parametrize("n_shards", [1, 3])
def test_wide_local_validator_trust(name, n_shards):
    """validator_trust (yumas.py:224, `W_clipped.sum(1) /
    W.sum(1)`) from miner-column shards: stage 3 sums Wc and Wn over each
    shard's tiles, the totals are added in shard order. One shard adds the
    tiles exactly as the unsharded finalize (bitwise); three shards
    re-associate the sum (within 1e-5)."""
    variant, par = CASES[name]
    W, S = _inputs(0x5EED47)
    params = _params(variant, par, W.shape[1])
    ref = engine.run(variant, params, W, S, want_hist=True, want=("Tv",))
    got = wide.run_wide_local(variant, params, W, S, n_shards, want_hist=True, want=("Tv",))
    torch.cuda.synchronize()
    _compare(got, ref, wide.column_ranges(M, n_shards))
    tv = got.extra["Tv"][0]
    if n_shards == 1:
        assert torch.equal(tv, ref.extra["Tv"])
    else:
        for t in got.extra["Tv"][1:]:
            assert torch.equal(t, tv)  # every shard holds the same totals
        assert_close(tv.cpu().numpy(), ref.extra["Tv"].cpu().numpy(), what="Tv")


@pytest.mark.gpu
@pytest.mark.parametrize("reset", [engine.RESET_ALWAYS, engine.RESET_IF_ZERO_CONSENSUS])
def test_wide_local_bond_reset(reset):
    variant = engine.VARIANT_YUMA3 if reset == engine.RESET_ALWAYS else engine.VARIANT_YUMA4
    W, S = _inputs(0x5EED44)
    params = _params(variant, {}, W.shape[1], reset=reset)
    ref = engine.run(variant, params, W, S, want_hist=True)
    got = wide.run_wide_local(variant, params, W, S, 3, want_hist=True)
    torch.cuda.synchronize()
    _compare(got, ref, wide.column_ranges(M, 3))
    # the reset really fired (on the shard that owns column 150): only that
    # column differs from a run without the reset
    plain = engine.run(variant, _params(variant, {}, W.shape[1]), W, S, want_hist=True)
    Bh, Bp = ref.B_hist.cpu().numpy(), plain.B_hist.cpu().numpy()
    assert not np.array_equal(Bh[2:, :, :, 150], Bp[2:, :, :, 150])
    np.testing.assert_array_equal(np.delete(Bh, 150, axis=3), np.delete(Bp, 150, axis=3))


@pytest.mark.gpu
def test_wide_local_against_oracle():
    from oracle import yuma_oracle as orc

    W, S = _inputs(0x5EED45, N=1)
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=True))
    params = [engine.make_params(engine.VARIANT_YUMA4, cfg)]
    got = wide.run_wide_local(engine.VARIANT_YUMA4, params, W, S, 3, want_hist=True)
    torch.cuda.synchronize()
    ref = orc.run("Yuma 4 (Rhef+relative bonds) - liquid alpha on", W[:, 0].numpy(), S[:, 0].numpy(), cfg)
    np.testing.assert_array_equal(torch.cat(got.C, dim=2)[:, 0].cpu().numpy(), ref["C"])
    assert_close(got.Dn[:, 0].cpu().numpy(), ref["Dn"], what="Dn")
    assert_close(torch.cat(got.B_hist, dim=3)[:, 0].cpu().numpy(), ref["B"], what="B")


def _wide_worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        variant, par = CASES[name]
        W, S = _inputs(0x5EED46)
        params = _params(variant, par, W.shape[1])
        cols = wide.column_ranges(M, world)[rank]
        res = wide.run_wide_distributed(variant, params, W[..., cols.start:cols.stop].contiguous(), S,
                                        M_total=M, want_hist=True)
        torch.cuda.synchronize()
        q.put((rank, res.Dn.cpu().numpy(), res.C[0].cpu().numpy(), res.I[0].cpu().numpy(),
               res.B_hist[0].cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["yuma3", "yuma4_liquid"])
def test_wide_distributed_two_ranks(name):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wide_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, *vals = q.get(timeout=100)
        got[r] = vals
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    variant, par = CASES[name]
    W, S = _inputs(0x5EED46)
    ref = engine.run(variant, _params(variant, par, W.shape[1]), W, S, want_hist=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got[0][0], got[1][0])  # every rank: the same dividends
    np.testing.assert_array_equal(np.concatenate([got[r][1] for r in range(world)], axis=2),
                                  ref.C.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate([got[r][3] for r in range(world)], axis=3),
                                  ref.B_hist.cpu().numpy())
    assert_close(got[0][0], ref.Dn.cpu().numpy(), what="Dn")
    assert_close(np.concatenate([got[r][2] for r in range(world)], axis=2), ref.I.cpu().numpy(), what="I")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rust", "yuma1_liquid", "yuma2"])
def test_wide_local_strip_scan_matches_unsharded(name):
    """The column-normalised strip scan (k_bonds_cn, subnets above 64
    validators) under miner-column shards: the bond recurrence normalises
    over validators only, so consensus and the bonds are bitwise those of the
    unsharded run; dividends add the shards' strip partials in shard order
    (within 1e-5)."""
    variant, par = CASES[name]
    Ew, Vw, Mw = 5, 136, 400
    W = torch.from_numpy(synth.weights(0x5EED9, Ew, 2, Vw, Mw))
    S = torch.from_numpy(synth.stakes(0x5EED9, Ew, 2, Vw, period=2))
    params = _params(variant, par, 2)
    ref = engine.run(variant, params, W, S, want_hist=True)
    got = wide.run_wide_local(variant, params, W, S, 3, want_hist=True)
    torch.cuda.synchronize()
    _compare(got, ref, wide.column_ranges(Mw, 3))


def _gather4_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = wide.dist_gather()
        widths = [3, 1, 4, 2]
        x = torch.arange(2 * widths[rank], dtype=torch.int32).reshape(2, widths[rank]) + 1000 * rank
        parts = g([x], widths)
        q.put((rank, [p.numpy() for p in parts]))
    finally:
        dist.destroy_process_group()


def test_dist_gather_four_ranks_uneven():
    """the padded all-gather with more than two ranks and
    uneven last dimensions (int32, as the liquid-alpha level exchange)."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    widths = [3, 1, 4, 2]
    for r in range(world):
        for k in range(world):
            exp = np.arange(2 * widths[k], dtype=np.int32).reshape(2, widths[k]) + 1000 * k
            np.testing.assert_array_equal(got[r][k], exp)


# c4's width plus three tiles: 1027 tiles cut into 257 + 257 + 257 + 256
E4, V4, M4 = 3, 256, 65536 + 64 * 3


def _c4_inputs():
    W = engine.synth_weights(0x5EED0004, E4, 1, V4, M4)
    S = torch.from_numpy(synth.stakes(0x5EED0004, E4, 1, V4, period=2)).to(W.device)
    return W, S


def _wide4_worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        variant, par = CASES[name]
        W, S = _c4_inputs()
        params = _params(variant, par, 1)
        cols = wide.column_ranges(M4, world)[rank]
        res = wide.run_wide_distributed(variant, params, W[..., cols.start:cols.stop].contiguous(), S,
                                        M_total=M4, want_hist=True)
        torch.cuda.synchronize()
        q.put((rank, res.Dn.cpu().numpy(), res.C[0].cpu().numpy(), res.I[0].cpu().numpy(),
               res.B_hist[0].cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["yuma4_liquid", "yuma1"])
def test_wide_distributed_four_ranks_uneven(name):
    """c4's wide subnet (256 x 65728: uneven shards) over
    four gloo ranks sharing the GPU — the padded dist_gather, the liquid-alpha
    level exchange and the shard-ordered sums with more than two ranks —
    bitwise equal to run_wide_local(..., 4) (the same stages and shard-order
    sums in one process); yuma1 runs its element-wise bond scan on the rank
    pass's column sums inside each shard."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_wide4_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in procs:
        r, *vals = q.get(timeout=200)
        got[r] = vals
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    variant, par = CASES[name]
    W, S = _c4_inputs()
    cols = wide.column_ranges(M4, world)
    assert len({len(c) for c in cols}) == 2  # uneven shards
    ref = wide.run_wide_local(variant, _params(variant, par, 1), W, S, world, want_hist=True)
    torch.cuda.synchronize()
    for r in range(world):
        np.testing.assert_array_equal(got[r][0], ref.Dn.cpu().numpy())  # every rank: the same dividends
        np.testing.assert_array_equal(got[r][1], ref.C[r].cpu().numpy())
        np.testing.assert_array_equal(got[r][2], ref.I[r].cpu().numpy())
        np.testing.assert_array_equal(got[r][3], ref.B_hist[r].cpu().numpy())
