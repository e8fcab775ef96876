"""Multi-process scenario sharding over torch.distributed (gloo, world_size 2).

CPU tests: the ranks use a CPU stand-in runner built on the oracle; what is
tested is the distribution logic (shard boundaries, per-rank parameter
selection, the rank-ordered gather). GPU tests: the same
two ranks run the HIP engine (two processes sharing one GPU), replicated and
shared-input (c3) sweeps, bitwise against the one-process run."""

import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import yuma_oracle as orc
from yuma_simulation._internal import synth
from yuma_simulation._internal.sharding import run_sharded, shard_range
from yuma_simulation._internal.yumas import SimulationHyperparameters, YumaConfig, YumaParams

VERSION = "Yuma 4 (Rhef+relative bonds) - liquid alpha on"


def oracle_runner(variant, configs, W, S, **_):
    """CPU stand-in with engine.run's signature/return shape."""
    outs = [orc.run(VERSION, W[:, j].numpy(), S[:, j].numpy(), cfg) for j, cfg in enumerate(configs)]
    return SimpleNamespace(
        Dn=torch.from_numpy(np.stack([o["Dn"] for o in outs], axis=1)),
        C=torch.from_numpy(np.stack([o["C"] for o in outs], axis=1)),
        I=torch.from_numpy(np.stack([o["I"] for o in outs], axis=1)),
        B_final=torch.from_numpy(np.stack([o["B"][-1] for o in outs])),
    )


def configs(n):
    return [YumaConfig(simulation=SimulationHyperparameters(kappa=0.4 + 0.05 * i),
                       yuma_params=YumaParams(liquid_alpha=True, bond_alpha=0.025 * (i + 1)))
            for i in range(n)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        E, V, M = 4, 8, 24
        W = torch.from_numpy(synth.weights(9, E, n_total, V, M))
        S = torch.from_numpy(synth.stakes(9, E, n_total, V, period=2))
        mine = shard_range(n_total, world, rank)
        res = run_sharded(4, configs(n_total), W[:, mine.start:mine.stop], S[:, mine.start:mine.stop],
                          n_total=n_total, runner=oracle_runner)
        q.put((rank, res.Dn.numpy(), res.C.numpy(), res.I.numpy(), list(res.local)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [5, 2])
def test_scenario_sharding_gloo_world2(n_total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # unsharded reference of the same scenarios
    E, V, M = 4, 8, 24
    W = synth.weights(9, E, n_total, V, M)
    S = synth.stakes(9, E, n_total, V, period=2)
    full = oracle_runner(4, configs(n_total), torch.from_numpy(W), torch.from_numpy(S))
    for rank, Dn, C, I, local in got:
        assert local == list(shard_range(n_total, world, rank))
        np.testing.assert_array_equal(Dn, full.Dn.numpy())  # every rank holds all scenarios
        np.testing.assert_array_equal(C, full.C.numpy())
        np.testing.assert_array_equal(I, full.I.numpy())


def test_shard_range_partitions():
    for n in range(0, 20):
        for world in range(1, 9):
            parts = [shard_range(n, world, r) for r in range(world)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


# ---------------------------------------------------------------------------
# GPU: the engine inside the ranks
# ---------------------------------------------------------------------------
GE, GV, GM = 6, 64, 512


def _engine_worker(rank, world, port, n_total, shared, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from yuma_simulation._internal import engine

        params = [engine.make_params(engine.VARIANT_YUMA4, c) for c in configs(n_total)]
        mine = shard_range(n_total, world, rank)
        W = engine.synth_weights(11, GE, 1 if shared else n_total, GV, GM)
        S = torch.from_numpy(synth.stakes(11, GE, 1 if shared else n_total, GV, period=2)).to(W.device)
        if not shared:
            W, S = W[:, mine.start:mine.stop].contiguous(), S[:, mine.start:mine.stop].contiguous()
        res = run_sharded(engine.VARIANT_YUMA4, params, W, S, n_total=n_total, shared_inputs=shared)
        torch.cuda.synchronize()
        q.put((rank, res.Dn.cpu().numpy(), res.C.cpu().numpy(), res.I.cpu().numpy(),
               res.B_final.cpu().numpy(), list(res.local)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("n_total,shared", [(5, False), (6, True)])
def test_engine_scenario_sharding_gloo_world2(n_total, shared):
    """run_sharded -> engine.run in each of two ranks (one GPU, two
    processes): every rank holds all scenarios' Dn / C / I after the gather
    and its own B_final, all bitwise equal to one engine call over every
    scenario in this process."""
    from yuma_simulation._internal import engine

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_engine_worker, args=(r, world, port, n_total, shared, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    params = [engine.make_params(engine.VARIANT_YUMA4, c) for c in configs(n_total)]
    W = engine.synth_weights(11, GE, 1 if shared else n_total, GV, GM)
    S = torch.from_numpy(synth.stakes(11, GE, 1 if shared else n_total, GV, period=2)).to(W.device)
    full = engine.run(engine.VARIANT_YUMA4, params, W, S, shared_inputs=shared)
    torch.cuda.synchronize()
    for rank, Dn, C, I, Bf, local in got:
        assert local == list(shard_range(n_total, world, rank))
        np.testing.assert_array_equal(Dn, full.Dn.cpu().numpy())
        np.testing.assert_array_equal(C, full.C.cpu().numpy())
        np.testing.assert_array_equal(I, full.I.cpu().numpy())
        np.testing.assert_array_equal(Bf, full.B_final[local[0]:local[-1] + 1].cpu().numpy())


def _timed_worker(rank, world, port, q):
    """bench.timed with a collective inside the step (c4's shard exchanges)
    and ranks of different speed: the clock ramp must end on the same step
    on every rank, or the ranks' collectives pair up wrongly and hang."""
    import sys
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), YUMA_BENCH_BACKEND="gloo")
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    import bench

    torch.cuda.synchronize = lambda *a, **k: None  # CPU-only rehearsal
    bench.PREWARM_S = 0.3
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = [0]

        def step():
            time.sleep(0.002 if rank == 0 else 0.02)  # rank 1 is 10x slower
            t = torch.ones(1)
            dist.all_reduce(t)
            n[0] += 1

        if rank == 1:
            time.sleep(0.5)  # ranks reach the timing at different moments
        elapsed = bench.timed(step, 2, 3, True, torch.device("cpu"))
        q.put((rank, n[0], elapsed))
    finally:
        dist.destroy_process_group()


def test_bench_timed_ranks_agree_on_step_count():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][1] == got[1][1]  # same number of steps on both ranks
    assert got[0][2] == got[1][2]  # the max over ranks, on every rank


# ---------------------------------------------------------------------------
# GPU: the RCCL (nccl backend) path on the one-GPU box, world size 1
# ---------------------------------------------------------------------------
def _nccl_worker(port, q):
    """A fresh process whose first GPU work is the nccl process group, as
    bench.py's N-rank path opens it (init_process_group("nccl", device_id)).
    Runs the wide subnet through run_wide_distributed (dist_gather's device
    branch: RCCL all-gathers of the per-shard partials) and the scenario
    gather of run_sharded, then the same work without the process group."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from yuma_simulation._internal import engine, sharding, wide

        assert dist.get_backend() == "nccl"
        E, V, M = 4, 64, 1024
        cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=True))
        params = [engine.make_params(engine.VARIANT_YUMA4, cfg)]
        W = engine.synth_weights(0x5EED0004, E, 1, V, M)
        S = torch.from_numpy(synth.stakes(0x5EED0004, E, 1, V, period=2)).to(W.device)
        got = wide.run_wide_distributed(engine.VARIANT_YUMA4, params, W, S, M_total=M, want_hist=True,
                                        want=("Tv",))
        # scenario sharding: 3 scenarios, this rank owns all; the rank-ordered
        # gather of the per-epoch results through RCCL
        n = 3
        p3 = [engine.make_params(engine.VARIANT_YUMA4, c) for c in configs(n)]
        W3 = engine.synth_weights(11, E, n, V, M)
        S3 = torch.from_numpy(synth.stakes(11, E, n, V, period=2)).to(W3.device)
        sh = sharding.run_sharded(engine.VARIANT_YUMA4, p3, W3, S3, n_total=n)
        gathered = sharding._gather_scenarios(sh.Dn, [n])
        torch.cuda.synchronize()
        dist.destroy_process_group()
        ref = wide.run_wide_local(engine.VARIANT_YUMA4, params, W, S, 1, want_hist=True, want=("Tv",))
        full = engine.run(engine.VARIANT_YUMA4, p3, W3, S3)
        torch.cuda.synchronize()
        q.put({
            "wide_Dn": torch.equal(got.Dn, ref.Dn),
            "wide_C": torch.equal(got.C[0], ref.C[0]),
            "wide_Bh": torch.equal(got.B_hist[0], ref.B_hist[0]),
            "wide_Tv": torch.equal(got.extra["Tv"][0], ref.extra["Tv"][0]),
            "wide_vs_unsharded": torch.equal(got.B_final[0], engine.run(
                engine.VARIANT_YUMA4, params, W, S).B_final),
            "sharded": all(torch.equal(getattr(sh, k), getattr(full, k)) for k in ("Dn", "C", "I", "B_final")),
            "gather": torch.equal(gathered, full.Dn) and gathered.is_cuda,
        })
    except Exception as e:  # reported to the parent, which fails the test
        import traceback

        q.put({"error": f"{type(e).__name__}: {e}\n{traceback.format_exc()}"})


@pytest.mark.gpu
def test_rccl_world1_wide_and_scenario_gather():
    """the nccl (RCCL) backend in a world-1 group on the
    one-GPU box — run_wide_distributed's all-gathers of row-sum / ΣC / ΣR /
    level / dividend / trust partials (dist_gather's device branch) and the
    scenario gather of run_sharded — bitwise equal to the in-process shard
    driver (run_wide_local(..., 1)), the unsharded engine and engine.run.
    Reference reductions replaced: yumas.py:411,436,445,475-476."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    assert all(res.values()), res
