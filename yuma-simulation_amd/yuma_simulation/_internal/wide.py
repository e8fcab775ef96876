"""Wide subnets sharded by miner column (BASELINE config c4:
256 validators x 65536 miners).

The reference runs a wide subnet exactly like a narrow one — one Yuma* call
per epoch (yumas.py:399 Yuma3 etc.) inside run_simulation
(simulation_utils.py:44-110). Every quantity that crosses miner columns in
that epoch step is a SUM over columns — row sums (yumas.py:186), sum C
(:211), sum R (:220), the dividends D (:261, :474, :589) — or a quantile of
C (:231-247, liquid alpha), and the bond recurrence is column-local. So each
process (one per GPU) owns a contiguous block of miner columns and runs the
whole E-epoch trajectory through the engine's five shard stages
(include/yuma_hip.h, yuma_shard_stage); between stages the per-shard
partials are all-gathered (RCCL over xGMI; gloo on CPU) and summed in shard
order, so every rank sees bit-identical totals and the result does not
depend on timing. Four small exchanges per run, independent of E:
[E,N,V] row sums, [E,N] sum C, [E,N] sum R (+ the [E,N,M] levels when a
scenario uses liquid alpha), [E,N,V] dividend partials (+ the [2,E,N,V] sums
of Wc and Wn when validator_trust, yumas.py:224, is requested). The level
exchange is SURVEY §8e's "all-gather of C" option (the quantised C as int32
levels, M_total x 4 B per slice): the same bytes as a 65536-bin histogram and
one exchange instead of a two-pass radix select.

The same orchestration drives several shards inside ONE process
(`run_wide_local`); `run_wide_distributed` is the one-shard-per-rank form.

Exactness. Every rank gets the same bits for any shard count's totals, but
those totals are added in shard order: ((shard0 + shard1) + shard2) ...,
where the unsharded engine adds the same 256-miner chunk sums strictly left
to right. The two orders give identical fp32 results whenever the partial
sums are exact -- the integer-valued synthetic weights of the benchmarks,
whose row sums stay below 2^24, are -- and that case is tested bit-for-bit
against the unsharded run (tests/test_wide.py, test_gpu_configs.py c4). On
generic float weights a row sum can differ by an ulp, which can move a
consensus decision inside the tie window (oracle.tie_columns); that case is
tested against the oracle: C exact outside the window, the rest within 1e-5
(test_gpu_configs.test_wide_float_weights_against_oracle).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch
import torch.distributed as dist

from . import engine

TILE = 64  # engine tile width: shards are cut on tile boundaries


def column_ranges(M: int, n_shards: int) -> list[range]:
    """Contiguous, balanced, tile-aligned column blocks (the first shards get
    one tile more when the tiles do not divide evenly)."""
    if n_shards < 1:
        raise ValueError("n_shards must be >= 1")
    tiles = -(-M // TILE)
    if tiles < n_shards:
        raise ValueError(f"{M} miners ({tiles} tiles of {TILE}) cannot be cut into {n_shards} shards")
    base, extra = divmod(tiles, n_shards)
    out, t0 = [], 0
    for r in range(n_shards):
        t1 = t0 + base + (1 if r < extra else 0)
        out.append(range(t0 * TILE, min(t1 * TILE, M)))
        t0 = t1
    return out


def shard_params(params: list, cols: range) -> list:
    """Per-shard copies of the parameter records: the bond-reset column
    (simulation_utils.py:62-88) becomes shard-local, or the reset is dropped
    on shards that do not own it; an all-columns reset stays on every shard."""
    out = []
    for p in params:
        q = type(p).from_buffer_copy(bytes(p))
        if q.reset_mode != engine.RESET_NONE and not q.flags & engine.FLAG_RESET_ALL_COLUMNS:
            if q.reset_index in cols:
                q.reset_index = q.reset_index - cols.start
            else:
                q.reset_mode = engine.RESET_NONE
                q.reset_index = 0
        out.append(q)
    return out


def ordered_sum(parts: list[torch.Tensor]) -> torch.Tensor:
    """Sum of the shards' partials in shard order (fixed association, so the
    total is the same bits on every rank and run)."""
    acc = parts[0].clone()
    for p in parts[1:]:
        acc = acc + p
    return acc


@dataclass
class WideResult:
    Dn: torch.Tensor                 # [E, N, V] (identical on every shard)
    C: list[torch.Tensor]            # per local shard [E, N, M_local]
    I: list[torch.Tensor]            # per local shard [E, N, M_local]
    B_final: list[torch.Tensor]      # per local shard [N, V, M_local]
    B_hist: list[torch.Tensor] | None
    cols: list[range]                # global columns of each local shard
    extra: dict


# gather(list of this process's per-shard tensors, widths) -> every shard's
# tensor in global shard order. widths: None when every shard's tensor has the
# same shape, else the last-dimension size of each global shard (known from
# column_ranges, so no size exchange is needed).
Gather = Callable[..., list[torch.Tensor]]


def _run_shards(variant: int, params: list, W_shards: list[torch.Tensor], S: torch.Tensor,
                cols: list[range], M_total: int, gather: Gather, all_cols: list[range], *,
                B_init: list[torch.Tensor] | None = None,
                Wprev_init: list[torch.Tensor] | None = None,
                want_hist: bool = False, want: tuple[str, ...] = ()) -> WideResult:
    """Drive the five shard stages over the LOCAL shards. `gather(list of this
    process's per-shard tensors)` returns every shard's tensor in global
    shard order (identity inside one process, an all-gather across ranks)."""
    dev = engine.device()
    k = len(W_shards)
    E, N, V, _ = W_shards[0].shape
    S = S.to(device=dev, dtype=torch.float32).contiguous()
    if S.shape != (E, N, V):
        raise ValueError(f"S shape {tuple(S.shape)} does not match W [E={E}, N={N}, V={V}]")
    if len(params) != N:
        raise ValueError("one parameter record per scenario is required")
    rust = variant == engine.VARIANT_RUST
    liquid = any(p.liquid_mode == engine.LIQUID_QUANTILE for p in params)
    f32 = dict(dtype=torch.float32, device=dev)
    sh = []
    for i in range(k):
        W = W_shards[i].to(device=dev, dtype=torch.float32).contiguous()
        M = W.shape[3]
        if W.shape[:3] != (E, N, V) or M != len(cols[i]):
            raise ValueError(f"shard {i}: W {tuple(W.shape)} does not match columns {cols[i]}")
        prm = engine.params_tensor(shard_params(params, cols[i]), dev)
        ws = torch.empty(max(engine.workspace_bytes(variant, N, E, V, M, "Tv" in want), 1),
                         dtype=torch.uint8, device=dev)
        out = {"Dn": torch.empty(E, N, V, **f32), "C": torch.empty(E, N, M, **f32),
               "I": torch.empty(E, N, M, **f32), "B_final": torch.empty(N, V, M, **f32)}
        if want_hist:
            out["B_hist"] = torch.empty(E, N, V, M, **f32)
        shapes = {"D": (E, N, V), "R": (E, N, M), "P": (E, N, M), "T": (E, N, M), "Tv": (E, N, V),
                  "Sn": (E, N, V), "bond_alpha": (E, N, M), "alpha_ab": (E, N, 2)}
        for name in want:
            if name not in shapes:
                raise ValueError(f"output {name!r} is not produced by a column shard")
            out[name] = torch.empty(shapes[name], **f32)
        if "T" in out and "P" not in out:
            out["P"] = torch.empty(shapes["P"], **f32)
        io = {"rowsum_part": torch.empty(E, N, V, **f32),
              "levels": torch.empty(E, N, M, dtype=torch.int32, device=dev),
              "rsum_part": torch.empty(E, N, **f32),
              "dsum_part": torch.empty(E, N, V, **f32)}
        if "Tv" in want:
            io["tv_part"] = torch.empty(2, E, N, V, **f32)
        if rust:
            io["csum_part_d"] = torch.empty(E, N, dtype=torch.float64, device=dev)
        else:
            io["csum_part"] = torch.empty(E, N, **f32)
        bi = None if B_init is None else B_init[i].to(**f32).contiguous()
        wp = None if Wprev_init is None else Wprev_init[i].to(**f32).contiguous()
        sh.append(dict(W=W, prm=prm, ws=ws, out=out, io=io, B_init=bi, Wprev=wp, col0=cols[i].start))

    def stage(n: int) -> None:
        for s in sh:
            engine.shard_stage(n, variant, s["prm"], s["W"], S, s["B_init"], s["Wprev"],
                               M_total=M_total, col0=s["col0"], io=s["io"], out=s["out"],
                               workspace=s["ws"])

    def reduce(name: str) -> torch.Tensor:
        return ordered_sum(gather([s["io"][name] for s in sh], None))

    stage(1)
    rowsum = reduce("rowsum_part")
    for s in sh:
        s["io"]["rowsum"] = rowsum
    stage(2)
    if rust:
        csum = reduce("csum_part_d")
        for s in sh:
            s["io"]["csum_d"] = csum
    else:
        csum = reduce("csum_part")
        for s in sh:
            s["io"]["csum"] = csum
    stage(3)
    rsum = reduce("rsum_part")
    tv = reduce("tv_part") if "Tv" in want else None
    levels_all = None
    if liquid:
        widths = [len(c) for c in all_cols]
        levels_all = torch.cat(gather([s["io"]["levels"] for s in sh], widths), dim=2).contiguous()
    for s in sh:
        s["io"]["rsum"] = rsum
        if tv is not None:
            s["io"]["tv"] = tv
        if levels_all is not None:
            s["io"]["levels_all"] = levels_all
    stage(4)
    dsum = reduce("dsum_part")
    for s in sh:
        s["io"]["dsum"] = dsum
    stage(5)
    extra = {name: [s["out"][name] for s in sh] for name in sh[0]["out"]
             if name not in ("Dn", "C", "I", "B_final", "B_hist")}
    extra["_keep"] = (sh, S)
    return WideResult(
        Dn=sh[0]["out"]["Dn"],
        C=[s["out"]["C"] for s in sh], I=[s["out"]["I"] for s in sh],
        B_final=[s["out"]["B_final"] for s in sh],
        B_hist=[s["out"]["B_hist"] for s in sh] if want_hist else None,
        cols=cols, extra=extra)


def run_wide_local(variant: int, params: list, W: torch.Tensor, S: torch.Tensor, n_shards: int,
                   **kw) -> WideResult:
    """All shards of a W [E,N,V,M] subnet inside this process (one GPU): the
    same stages and the same shard-ordered sums as the distributed run."""
    M = W.shape[3]
    cols = column_ranges(M, n_shards)
    W_shards = [W[..., c.start:c.stop] for c in cols]
    B_init = kw.pop("B_init", None)
    Wprev = kw.pop("Wprev_init", None)
    if B_init is not None:
        kw["B_init"] = [B_init[..., c.start:c.stop] for c in cols]
    if Wprev is not None:
        kw["Wprev_init"] = [Wprev[..., c.start:c.stop] for c in cols]
    return _run_shards(variant, params, W_shards, S, cols, M, lambda xs, widths=None: xs, cols, **kw)


def dist_gather(group=None) -> Gather:
    """All-gather of one tensor per rank (RCCL over xGMI under the nccl
    backend; through host memory under gloo), ranks in order. Shapes are known
    up front — equal on every rank, or differing only in the last dimension
    by the caller's `widths` (uneven column shards) — so one collective per
    exchange, no size exchange and no host synchronisation under nccl."""
    world = dist.get_world_size(group)
    cpu = dist.get_backend(group) == "gloo"

    def gather(xs: list[torch.Tensor], widths: list[int] | None = None) -> list[torch.Tensor]:
        (x,) = xs
        dev = x.device
        if widths is not None:
            if len(widths) != world:
                raise ValueError(f"{len(widths)} widths for {world} ranks")
            width = max(widths)
            src = torch.zeros(*x.shape[:-1], width, dtype=x.dtype, device=dev)
            src[..., : x.shape[-1]] = x
        else:
            src = x.contiguous()
        if cpu:
            src = src.cpu()
        parts = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(parts, src, group=group)
        if widths is not None:
            parts = [p[..., :w] for p, w in zip(parts, widths)]
        return [p.to(dev) for p in parts]

    return gather


def run_wide_distributed(variant: int, params: list, W_local: torch.Tensor, S: torch.Tensor, *,
                         M_total: int, group=None, **kw) -> WideResult:
    """This rank's shard (columns column_ranges(M_total, world)[rank]) of a
    wide subnet; one process per GPU."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cols = column_ranges(M_total, world)[rank]
    if W_local.shape[3] != len(cols):
        raise ValueError(f"rank {rank} holds {W_local.shape[3]} columns, its shard is {cols}")
    for key in ("B_init", "Wprev_init"):
        if kw.get(key) is not None:
            kw[key] = [kw[key]]
    return _run_shards(variant, params, [W_local], S, [cols], M_total, dist_gather(group),
                       column_ranges(M_total, world), **kw)
