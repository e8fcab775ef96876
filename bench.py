"""Benchmark: scenario-epochs/s of the Yuma epoch engine on MI355X.

Workload (BASELINE.json configs[1], "c2"): one subnet of 256 validators x
4096 miners run for 1000 epochs with "Yuma 3 (Rhef)"; synthetic exactness-
friendly inputs (yuma_simulation._internal.synth), resident in HBM before the
timed region. One *step* = one engine call over the whole 1000-epoch
trajectory from an empty bond state, writing every epoch's bond state
(run_simulation's bonds_per_epoch), consensus, incentive and normalised
dividends — the epoch-step contract of SURVEY §8d.

Multi-GPU (torchrun, one process per GPU): scenario sharding — every rank runs
its own subnet (its own seed), no data-path collective; weak scaling.

Prints ONE JSON line (rank 0) with the driver's fields plus `roofline`
(dominant kernel, algorithmic bytes / measured device time from HIP events)
and `cpu_baseline` (the numpy oracle on a bounded sample, host cores).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "yuma-simulation_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "scenario-epochs/sec (256V x 4096M) at 1/8 GPUs; % of HBM peak GB/s"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def phase_bytes(phase: str, V: int, M: int, variant: int, liquid: bool, hist: bool, chunk: int) -> float:
    """Algorithmic HBM bytes one phase must move per scenario-epoch (each input
    read once, each output written once). DESIGN.md §Roofline tabulates them."""
    tiles = (M + 63) // 64
    VM = V * M
    colnorm = variant <= 2
    table = {
        "rowsum": 4 * VM + 4 * V + 8 * V,
        "consensus": 4 * VM + 8 * V + 8 * M,
        "quantise": 8 * M + 8 * M + (4 * M if liquid else 0),
        "rank": 4 * VM + 8 * V + 4 * M + 4 * M + 4 * tiles,
        "incentive": 4 * M + 4 * tiles + 4 * M,
        "bonds": (4 * VM + 8 * V + 4 * M + (4 * M if colnorm else 0) + (4 * M if liquid else 0)
                  + (4 * VM if hist else 0) + 4 * V * tiles + 8 * VM / max(chunk, 1)),
        "finalize": 4 * V * tiles + 4 * V + 4 * V,
        # one W read; writes rs, S/sum S, C_raw (f64), C, levels, R, tile sums
        "phase1_fused": 4 * VM + 4 * V + 8 * V + 8 * M + 4 * M + 4 * M + 4 * M + 4 * tiles,
        "liquid": (4 * M + 4 * M + 4 * M) if liquid else 8 * M,
    }
    return float(table[phase])


def contract_bytes(V: int, M: int, variant: int) -> float:
    """SURVEY §8d epoch-step contract: read W_t, B_{t-1}, S_t; write B_t, Dn_t,
    C_t, I_t (Yuma2 adds W_prev)."""
    b = 4 * (3 * V * M + 2 * V + 2 * M)
    return float(b + (4 * V * M if variant == 2 else 0))


def cpu_baseline(version: str, V: int, M: int, epochs: int, ring: int, seed: int) -> dict:
    """The numpy oracle (oracle/yuma_oracle.py, a port of the reference
    algorithm) on `epochs` epochs of the same workload, one host core."""
    from oracle import yuma_oracle as orc
    from yuma_simulation._internal import synth
    from yuma_simulation._internal.yumas import YumaConfig

    Wr = synth.weights(seed, ring, 1, V, M)[:, 0]
    S = synth.stakes(seed, epochs, 1, V)[:, 0]
    W = np.stack([Wr[e % ring] for e in range(epochs)])
    t0 = time.perf_counter()
    orc.run(version, W, S, YumaConfig())
    dt = time.perf_counter() - t0
    return {
        "value": round(epochs / dt, 3),
        "unit": "scenario-epochs/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{epochs} epochs of {version} at {V}x{M} ({ring} distinct synthetic W epochs cycled), "
                  f"vectorised numpy oracle, 1 thread, {dt:.1f} s",
    }


def load_traffic(cfg: dict, dominant: str):
    """HBM bytes per launch from committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), if they were
    collected on this exact workload."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f)
    if rec.get("workload") != cfg:
        return None
    k = rec.get("kernels", {}).get(dominant)
    return None if k is None else k.get("hbm_bytes_per_scenario_epoch")


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--validators", type=int, default=256)
    ap.add_argument("--miners", type=int, default=4096)
    ap.add_argument("--scenarios", type=int, default=1, help="scenarios per GPU")
    ap.add_argument("--version", default="Yuma 3 (Rhef)")
    ap.add_argument("--liquid", action="store_true")
    ap.add_argument("--no-history", action="store_true", help="do not write every epoch's bond state")
    ap.add_argument("--chunk", type=int, default=0, help="epochs per phase-1 batch (0 = engine default)")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0002)
    ap.add_argument("--cpu-epochs", type=int, default=160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-reps", type=int, default=3)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from yuma_simulation._internal import engine, synth
    from yuma_simulation._internal.simulation_utils import resolve_version
    from yuma_simulation._internal.yumas import YumaConfig, YumaParams

    dev = engine.device()
    E, V, M, N = args.epochs, args.validators, args.miners, args.scenarios
    variant, _ = resolve_version(args.version)
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=args.liquid))
    params = [engine.make_params(variant, cfg) for _ in range(N)]
    liquid = params[0].liquid_mode != engine.LIQUID_OFF
    hist = not args.no_history
    seed = args.seed + 7919 * rank  # each rank simulates its own subnet(s)

    # inputs resident in HBM before timing
    W = engine.synth_weights(seed, E, N, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, N, V)).to(dev)
    out = {"Dn": torch.empty(E, N, V, device=dev), "C": torch.empty(E, N, M, device=dev),
           "I": torch.empty(E, N, M, device=dev), "B_final": torch.empty(N, V, M, device=dev)}
    if hist:
        out["B_hist"] = torch.empty(E, N, V, M, device=dev)
    ws = torch.empty(engine.workspace_bytes(variant, N, E, V, M, False), dtype=torch.uint8, device=dev)
    chunk = args.chunk

    def step():
        return engine.run(variant, params, W, S, want_hist=hist, out=out, workspace=ws, chunk_epochs=chunk)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_units = float(E) * N * world * args.steps
    value = total_units / elapsed

    # per-phase device time from HIP events on the launch stream (separate,
    # untimed passes of the same step)
    phases = np.zeros(len(engine.PHASES))
    for _ in range(args.profile_reps):
        buf = [0.0] * len(engine.PHASES)
        engine.run(variant, params, W, S, want_hist=hist, out=out, workspace=ws, chunk_epochs=chunk,
                   phase_ms=buf)
        phases += np.array(buf)
    phases /= args.profile_reps
    eff_chunk = chunk if 0 < chunk <= E else E
    units = E * N
    phase_info = {}
    for i, name in enumerate(engine.PHASES):
        b = phase_bytes(name, V, M, variant, liquid, hist, eff_chunk) * units
        phase_info[name] = {"ms": round(float(phases[i]), 4),
                            "GBps": round(b / (phases[i] * 1e-3) / 1e9, 1) if phases[i] > 0 else None}
    dom = int(np.argmax(phases))
    dom_name = engine.PHASES[dom]
    dom_bytes = phase_bytes(dom_name, V, M, variant, liquid, hist, eff_chunk) * units
    achieved = dom_bytes / (phases[dom] * 1e-3) / 1e9
    workload = {"workload": f"c2: single subnet {V}V x {M}M x {E} epochs, {args.version}"
                            + (" liquid" if liquid else ""),
                "V": V, "M": M, "epochs": E, "scenarios_per_gpu": N, "version": args.version,
                "bond_history": hist, "parallelism": f"scenario-sharded x{world}" if world > 1 else "single GPU"}
    traffic = load_traffic({k: workload[k] for k in ("V", "M", "epochs", "version", "bond_history")}, dom_name)

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "scenario-epochs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (integer-valued weights, stakes summing to 2^20; SURVEY §8d generator)",
        "config": workload,
        "roofline": {
            "bound": "hbm",
            "kernel": f"k_{dom_name}",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
        },
        "contract_GBps": round(value / world * contract_bytes(V, M, variant) / 1e9, 1),
        "phases": phase_info,
    }
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.version, V, M, args.cpu_epochs, 16, args.seed)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
