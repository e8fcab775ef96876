"""Multi-GPU execution: one process per GPU over torch.distributed (RCCL on
ROCm, gloo for CPU tests). SURVEY §8e.

Scenario sharding (configs c2 replicas, c3 sweeps, c5 sheet): scenarios are
independent, so each rank runs a contiguous block of them through the engine
with NO collective on the data path. Only the final per-epoch results
(normalised dividends, consensus, incentives — [E, N, V|M], small) are
all-gathered at the end when the caller wants them everywhere.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int) -> range:
    """Contiguous, balanced block of scenario indices owned by `rank`
    (the first n_total % world ranks get one extra)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


@dataclass
class ShardedResult:
    Dn: torch.Tensor  # [E, N_total, V] (gathered) or [E, n_local, V]
    C: torch.Tensor   # [E, N_total, M] or local
    I: torch.Tensor   # [E, N_total, M] or local
    B_final: torch.Tensor  # [n_local, V, M] — bond state stays on its GPU
    local: range


def _gather_scenarios(x: torch.Tensor, counts: list[int], group=None) -> torch.Tensor:
    """All-gather [E, n_local, ...] blocks of uneven size into [E, N_total, ...]
    in rank order (deterministic)."""
    world = len(counts)
    width = max(counts)
    pad = list(x.shape)
    pad[1] = width
    buf = torch.zeros(pad, dtype=x.dtype, device=x.device)
    buf[:, : x.shape[1]] = x
    if dist.get_backend(group) == "gloo":  # gloo gathers through host memory
        buf = buf.cpu()
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[:, :c] for p, c in zip(parts, counts)], dim=1).to(x.device)


def run_sharded(variant: int, params_all: list, W_local: torch.Tensor, S_local: torch.Tensor, *,
                n_total: int, gather: bool = True, group=None, runner=None, **run_kwargs) -> ShardedResult:
    """Run this rank's scenarios. W_local [E, n_local, V, M], S_local
    [E, n_local, V] hold exactly the scenarios of shard_range(n_total, world,
    rank) — or, with shared_inputs=True (a parameter sweep over one subnet,
    config c3), the one trajectory [E, 1, V, M] / [E, 1, V] every scenario
    reads; params_all has one record per GLOBAL scenario. `runner` defaults
    to engine.run (tests pass a CPU stand-in with the same signature)."""
    if runner is None:
        from yuma_simulation._internal import engine

        runner = engine.run
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mine = shard_range(n_total, world, rank)
    n_in = 1 if run_kwargs.get("shared_inputs") else len(mine)
    if W_local.shape[1] != n_in or S_local.shape[1] != n_in:
        raise ValueError(f"rank {rank} holds {W_local.shape[1]} scenarios, shard is {len(mine)}")
    res = runner(variant, [params_all[i] for i in mine], W_local, S_local, **run_kwargs)
    Dn, C, I = res.Dn, res.C, res.I
    if gather and world > 1:
        counts = [len(shard_range(n_total, world, r)) for r in range(world)]
        Dn = _gather_scenarios(Dn, counts, group)
        C = _gather_scenarios(C, counts, group)
        I = _gather_scenarios(I, counts, group)
    return ShardedResult(Dn, C, I, res.B_final, mine)
