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

Other BASELINE.json configs (`--config`, not what the driver runs):
  c3  batched parameter sweep: 512 scenarios per GPU of 256 x 4096 over the
      bond_alpha x kappa x liquid x (alpha_low, alpha_high) grid, Yuma 4;
  c4  wide subnet 256 x 65536, miner columns sharded across the ranks
      (RCCL all-gathers of per-shard partials between the engine's stages);
  c5  the full dividend sheet (4 bond penalties x 14 cases x 9 versions =
      504 runs) through generate_total_dividends_tables.

Prints ONE JSON line (rank 0) with the driver's fields plus
  roofline      SURVEY §8d step roofline: achieved = scenario-epochs/s per GPU x
                BYTES(V,M) (the fp32 epoch-step contract, 12,617,728 B at
                256 x 4096), frac = achieved / 8 TB/s; traffic = the rocprofv3
                FETCH_SIZE + WRITE_SIZE bytes of one step (committed PMC passes of
                this exact workload, profiles/r05/pmc_traffic.json), and
                roofline.kernel = the dominant kernel (k_bonds_elem at c2):
                algorithmic bytes per launch / its HIP-event launch time;
  cpu_baseline  the torch-CPU restatement of the epoch (oracle/torch_cpu.py,
                bit-identical to the reference goldens) on the host cores of
                this box: vectorised (value) and reference-structured (per-column
                Python bisection, as yumas.py runs it);
  also          (default c2 run) the same line's numbers for "Yuma 4 liquid",
                the second c2 version of SURVEY §7, on the same resident inputs.

`--gpus N` without torchrun re-launches itself under torch.distributed.run
with N local ranks (before anything touches a GPU).
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


def phase_bytes(phase: str, V: int, M: int, variant: int, liquid: bool, hist: bool, chunk: int,
                wshare: int = 1) -> float:
    """Algorithmic HBM bytes one phase must move per scenario-epoch (each input
    read once, each output written once). DESIGN.md §Roofline tabulates them.
    wshare: scenarios reading one shared input trajectory (the c3 sweep): W
    and the per-epoch row sums are read once per input epoch for all of them,
    so their bytes are divided among the wshare scenarios."""
    tiles = (M + 63) // 64
    # dividend partials per (slice, validator): 16-miner strips (YumaRust's
    # column-normalised strip scan), quads of 64-miner tiles (the wide history
    # scan and the history-less one-row scan), else one per tile (the sweep scan)
    if variant == 0:
        ptiles = (M + 15) // 16
    elif wshare == 1 and (not hist or M >= 1024):
        ptiles = (tiles + 3) // 4
    else:
        ptiles = tiles
    VM = V * M
    colnorm = variant <= 2
    w = 4 * VM / wshare
    table = {
        "consensus": w + 8 * V + 8 * M,
        "quantise": 8 * M + 8 * M + (4 * M if liquid else 0),
        # Yuma / Yuma2 also write the bond column sums csb [M] and csr [M]
        "rank": w + 8 * V + 4 * M + 4 * M + 4 * tiles + (8 * M if variant in (1, 2) else 0),
        "rowsum": w + (4 * V + 8 * V + 16 * V) / wshare,
        "incentive": 4 * M + 4 * tiles + 4 * M,
        # column-normalised variants read C and a column sum per miner (Yuma /
        # Yuma2: csb and its screened reciprocal csr, 12 B; YumaRust: its rank R, 8 B)
        "bonds": (w + 8 * V + 4 * M + ((12 if variant in (1, 2) else 8) * M if colnorm else 0)
                  + (4 * M if liquid else 0)
                  + (4 * VM if hist else 0) + 4 * V * ptiles + 8 * VM / max(chunk, 1)),
        "finalize": 4 * V * ptiles + 4 * V + 4 * V,
    }
    return float(table[phase])


PHASE_KERNELS = {"rowsum": "k_rowsum", "consensus": "k_consensus_w", "quantise": "k_quantise",
                 "rank": "k_rank_s", "incentive": "k_incentive", "finalize": "k_finalize"}


def kernel_of(phase: str, variant: int, shared: bool = False, V: int = 256, M: int = 4096,
              N: int = 1) -> str:
    """The kernel that runs a phase (as rocprofv3 names it) for run outputs:
    the bond scan is k_bonds_elem for Yuma 3/4 (k_bonds_grp for a sweep over
    one shared input trajectory) and, above 64 validators, for Yuma 1 / 2
    (the rank pass forms their bond column sums); YumaRust's strip scan
    k_bonds_cn above 64 validators; k_bonds on 64-miner tiles below."""
    if phase == "bonds":
        if variant >= 3:
            return "k_bonds_grp" if shared and N > 1 else "k_bonds_elem"
        if variant in (1, 2) and V > 64:
            return "k_bonds_elem"
        return "k_bonds_cn" if V > 64 and M % 4 == 0 else "k_bonds"
    if phase == "consensus" and 64 < V <= 256 and M % 4 == 0 and not shared:
        return "k_consensus_p"  # 128-byte row segments (wave pairs; run outputs)
    if phase == "rank" and ((variant in (1, 2) and V > 64) or M >= 16384):
        return "k_rank_sw"  # 256-miner column blocks (bond column sums; wide subnets)
    return PHASE_KERNELS[phase]


TRAFFIC_JSON = os.path.join(ROOT, "profiles", "r06", "pmc_traffic.json")
SQ_JSON = os.path.join(ROOT, "profiles", "r06", "sq_valu.json")


def engine_build_id() -> str:
    from yuma_simulation._internal import engine

    return engine.build_id()


def _matching_record(path: str, key: dict) -> dict | None:
    """The committed counter record of this exact workload measured on THIS
    library build (record build_id == yuma_build_id()), else None: a record
    from another build describes other kernels and is never paired with this
    run's timings."""
    try:
        with open(path) as f:
            records = json.load(f)
    except (OSError, ValueError):
        return None
    for rec in records:
        wl = rec.get("workload", {})
        if all(wl.get(k) == v for k, v in key.items()):
            return rec if rec.get("build_id") == engine_build_id() else None
    return None
VALU_PEAK_GINST = 1024 * 2.4 / 2  # G wave64 VALU instructions/s: 1024 SIMDs, 2 cycles each, 2.4 GHz


def load_sq(key: dict) -> dict | None:
    """Per-kernel SQ counts per launch (SQ_INSTS_VALU, ...) of the committed SQ
    pass of this exact workload on this library build (tools/sq_summary.py), or None."""
    rec = _matching_record(SQ_JSON, key)
    if rec is None:
        return None
    return {k: dict(v["counters"], commit=rec.get("commit"), build_id=rec.get("build_id"))
            for k, v in rec["kernels"].items()}


def load_traffic(key: dict) -> dict | None:
    """Per-kernel HBM bytes per scenario-epoch (FETCH_SIZE + WRITE_SIZE,
    corrected) of the committed PMC passes of this exact workload on this
    library build, or None."""
    rec = _matching_record(TRAFFIC_JSON, key)
    if rec is None:
        return None
    return {k: float(v["hbm_bytes_per_scenario_epoch"]) for k, v in rec["kernels"].items()}


def contract_bytes(V: int, M: int, variant: int) -> float:
    """SURVEY §8d epoch-step contract: read W_t, B_{t-1}, S_t; write B_t, Dn_t,
    C_t, I_t (Yuma2 adds W_prev)."""
    b = 4 * (3 * V * M + 2 * V + 2 * M)
    return float(b + (4 * V * M if variant == 2 else 0))


def host_cpu() -> dict:
    """The host this runs on: lscpu model, os.cpu_count(), the CPUs this
    process may use, and the torch thread count the CPU baseline uses
    (the process's CPU share, capped by OMP_NUM_THREADS when the scheduler
    sets it: a 1-GPU box exposes the whole machine's CPUs to os.cpu_count()
    but grants each GPU a share)."""
    import subprocess

    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    if model is None and os.path.exists("/proc/cpuinfo"):
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    total = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    threads = usable
    omp = os.environ.get("OMP_NUM_THREADS", "")
    share = "every usable CPU"
    if omp.isdigit() and int(omp) > 0 and int(omp) < usable:
        threads = int(omp)
        share = (f"this process's CPU share: the GPU scheduler grants each GPU OMP_NUM_THREADS={omp} of the "
                 f"host's {usable} usable CPUs (os.cpu_count() counts the whole host)")
    return {"model": model, "cpu_count": total, "usable": usable, "threads": threads, "share": share}


def cpu_baseline(variant: str, W_dev, S_dev, cfgs: list, seconds: float, warmup: int, structured_epochs: int,
                 label: str, ring: int = 64) -> dict:
    """SURVEY §8d CPU baseline: oracle/torch_cpu.py (the epoch restated in torch
    CPU ops, bit-identical to the reference goldens) on the host cores, over
    the SAME resident inputs (the first `ring` epochs copied back from HBM and
    cycled). value = the vectorised form (all columns' bisections per
    iteration, torch intra-op threads), timed for about `seconds`;
    `structured` = the reference's own loop structure (one Python bisection
    per miner column, yumas.py:197-209), `structured_epochs` epochs."""
    from oracle import torch_cpu as tc

    host = host_cpu()
    torch.set_num_threads(host["threads"])
    n_sc = len(cfgs)
    ring = min(ring, W_dev.shape[0])
    if W_dev.shape[1] == 1 and n_sc > 1:  # one shared trajectory (the c3 sweep)
        W = W_dev[:ring, :1].cpu().expand(-1, n_sc, -1, -1)
        S = S_dev[:ring, :1].cpu().expand(-1, n_sc, -1)
    else:
        W = W_dev[:ring, :n_sc].cpu()
        S = S_dev[:ring, :n_sc].cpu()

    key = tc.state_key(variant)

    def rate(mode: str, n_warm: int, max_epochs: int, budget: float) -> tuple[float, int, float]:
        B = [None] * n_sc
        Wp = [None] * n_sc  # Yuma 2: the previous epoch's normalised W

        def one(t: int, j: int, cfg) -> None:
            r = tc.epoch(variant, W[t % ring, j], S[t % ring, j], B[j], cfg, consensus=mode, W_prev=Wp[j])
            B[j] = r[key]
            if variant == "yuma2":
                Wp[j] = r["weight"]

        for t in range(n_warm):
            for j, cfg in enumerate(cfgs):
                one(t, j, cfg)
        t0 = time.perf_counter()
        n = 0
        while n < max_epochs and (n == 0 or time.perf_counter() - t0 < budget):
            t = n_warm + n
            for j, cfg in enumerate(cfgs):
                one(t, j, cfg)
            n += 1
        dt = time.perf_counter() - t0
        return n * n_sc / dt, n, dt

    vec, vn, vdt = rate("vectorised", warmup, 100000, seconds)
    st = None
    if structured_epochs > 0:
        st = rate("structured", 1, structured_epochs, float("inf"))
    return {
        "value": round(vec, 3),
        "unit": "scenario-epochs/s",
        "cores": host["threads"],
        "kind": "port",
        "sample": (f"{label}: oracle/torch_cpu.py vectorised, {warmup} warm-up + {vn} timed epochs x {n_sc} "
                   f"scenario(s) cycling the first {ring} resident epochs ({vdt:.1f} s), torch {host['threads']} "
                   f"threads on {host['model']} ({host['share']}); "
                   f"bit-identical to the reference goldens (tests/test_oracle_golden.py)"),
        "structured": None if st is None else {
            "value": round(st[0], 4), "unit": "scenario-epochs/s", "cores": 1,
            "sample": f"reference-structured per-column Python bisection, 1 warm-up + {st[1]} timed epochs x "
                      f"{n_sc} scenario(s) ({st[2]:.1f} s)"},
        "host": host,
    }


PREWARM_S = 1.0
# torch.distributed backend of the N-rank run: "nccl" (RCCL over xGMI, one GPU
# per rank); "gloo" only to rehearse the multi-rank path on a one-GPU box
BACKEND = os.environ.get("YUMA_BENCH_BACKEND", "nccl")


def timed(step, warmup: int, steps: int, dist: bool, dev) -> float:
    """An untimed clock ramp (steps repeated for PREWARM_S seconds: an idle
    MI355X takes ~6 c2 steps to reach its steady clocks, profiles/r03/c2y3
    kernel_trace.csv), W untimed warmups, then K steps between barrier +
    synchronize; the max over ranks of the elapsed wall time."""
    t_end = time.perf_counter() + PREWARM_S
    while True:
        for _ in range(8):
            step()
        torch.cuda.synchronize()
        done = time.perf_counter() >= t_end
        if dist:
            # every rank must run the same number of steps: a step may hold
            # collectives (c4's shard exchanges), so the ranks agree on when
            # the ramp ends
            import torch.distributed as tdist

            f = torch.tensor([1.0 if done else 0.0], device="cpu" if BACKEND == "gloo" else dev)
            tdist.all_reduce(f, op=tdist.ReduceOp.MAX)
            done = bool(f.item() > 0)
        if done:
            break
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        import torch.distributed as tdist

        tdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device="cpu" if BACKEND == "gloo" else dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def base_line(args, world: int, value: float, unit: str, elapsed: float, scaling: str, config: dict) -> dict:
    return {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (integer-valued weights, stakes summing to 2^20; SURVEY \u00a78d generator)",
        "config": config,
        # the library's source identity; counter-derived fields (traffic, the
        # c3 VALU roofline) are filled only from records of this same build
        "engine_build_id": engine_build_id(),
    }


SWEEP_BOND_ALPHA = [0.01 + (0.5 - 0.01) * i / 15 for i in range(16)]
SWEEP_KAPPA = [0.3 + (0.7 - 0.3) * i / 15 for i in range(16)]
SWEEP_ALPHAS = [(lo, hi) for lo in (0.6, 0.65, 0.7, 0.75) for hi in (0.9, 0.99)]


def sweep_config(g: int):
    """Scenario g of the c3 grid (SURVEY \u00a78d): 16 bond_alpha x 16 kappa x
    2 liquid x 8 (alpha_low, alpha_high) = 4096 scenarios."""
    from yuma_simulation._internal.yumas import SimulationHyperparameters, YumaConfig, YumaParams

    lo, hi = SWEEP_ALPHAS[(g // 512) % 8]
    return YumaConfig(simulation=SimulationHyperparameters(kappa=SWEEP_KAPPA[(g // 16) % 16]),
                      yuma_params=YumaParams(bond_alpha=SWEEP_BOND_ALPHA[g % 16],
                                             liquid_alpha=bool((g // 256) % 2),
                                             alpha_low=lo, alpha_high=hi))


def consensus_classes(params: list) -> int:
    """Scenarios of a shared-input run whose consensus the engine computes
    once (k_classes: equal kappa bits, trip count and histogram switch)."""
    import struct

    return len({(struct.pack("<f", p.kappa), p.bisect_iters, p.flags & 1) for p in params})


def engine_line(args, variant: int, params: list, W, S, world: int, dist: bool, workload: dict,
                shared: bool = False) -> dict:
    """Time one engine configuration on resident inputs and build its line:
    the step (graph replay of the whole E-epoch run), per-phase HIP-event
    device time, the §8d step roofline and the dominant kernel's roofline."""
    from yuma_simulation._internal import engine

    dev = W.device
    E, _, V, M = W.shape
    N = len(params)
    liquid = any(p.liquid_mode != engine.LIQUID_OFF for p in params)
    hist = not args.no_history
    out = {"Dn": torch.empty(E, N, V, device=dev), "C": torch.empty(E, N, M, device=dev),
           "I": torch.empty(E, N, M, device=dev), "B_final": torch.empty(N, V, M, device=dev)}
    if hist:
        out["B_hist"] = torch.empty(E, N, V, M, device=dev)
    ws = torch.empty(engine.workspace_bytes(variant, N, E, V, M, False), dtype=torch.uint8, device=dev)
    chunk = args.chunk
    graph = None
    if args.no_graph:
        def step():
            return engine.run(variant, params, W, S, want_hist=hist, out=out, workspace=ws, chunk_epochs=chunk,
                              shared_inputs=shared)
    else:
        # the whole E-epoch run captured once into a HIP graph (yuma_graph_create);
        # each timed step is one replay of it over the same resident inputs
        graph = engine.RunGraph(variant, params, W, S, want_hist=hist, out=out, workspace=ws, chunk_epochs=chunk,
                                shared_inputs=shared)
        step = graph.launch

    elapsed = timed(step, args.warmup, args.steps, dist, dev)
    units = E * N  # scenario-epochs per step per GPU
    value = float(units) * world * args.steps / elapsed

    # per-phase device time from HIP events recorded on the launch stream
    # (yuma_run_profiled: separate, untimed runs of the same step)
    phases = np.zeros(len(engine.PHASES))
    for _ in range(args.profile_reps):
        buf = [0.0] * len(engine.PHASES)
        engine.run(variant, params, W, S, want_hist=hist, out=out, workspace=ws, chunk_epochs=chunk, phase_ms=buf,
                   shared_inputs=shared)
        phases += np.array(buf)
    phases /= args.profile_reps
    if graph is not None:
        graph.close()
    eff_chunk = chunk if 0 < chunk <= E else E
    launches = -(-E // eff_chunk)  # launches of each phase kernel per step
    wshare = N if shared else 1
    phase_info = {}
    for i, name in enumerate(engine.PHASES):
        kname = kernel_of(name, variant, shared, V, M, N)
        if phases[i] <= 0:
            continue
        b = phase_bytes(name, V, M, variant, liquid, hist, eff_chunk, wshare) * units
        phase_info[name] = {"kernel": kname, "ms": round(float(phases[i]), 4),
                            "GBps": round(b / (phases[i] * 1e-3) / 1e9, 1)}
    dom_name = max(phase_info, key=lambda k: phase_info[k]["ms"])
    dom = engine.PHASES.index(dom_name)
    dom_kernel = kernel_of(dom_name, variant, shared, V, M, N)
    dom_bytes = phase_bytes(dom_name, V, M, variant, liquid, hist, eff_chunk, wshare) * units / launches
    dom_ms = float(phases[dom]) / launches
    k_achieved = dom_bytes / (dom_ms * 1e-3) / 1e9

    contract = contract_bytes(V, M, variant)
    per_gpu = value / world
    equivalent = per_gpu * contract / 1e9
    key = {k: workload[k] for k in ("V", "M", "epochs", "scenarios_per_gpu", "version", "bond_history")}
    pmc = load_traffic(key)
    traffic = None if pmc is None else round(sum(pmc.values()) * units)
    line = base_line(args, world, value, "scenario-epochs/s", elapsed, "weak", workload)
    kernel = {
        "name": dom_kernel,
        "launches_per_step": launches,
        "avg_ms": round(dom_ms, 4),
        "bytes_per_launch": dom_bytes,
        "achieved": round(k_achieved, 1),
        "frac": round(k_achieved / HBM_PEAK_GBPS, 4),
        "traffic": None if pmc is None or dom_kernel not in pmc else round(pmc[dom_kernel] * units / launches),
        "timing": "HIP events on the launch stream around the kernel (yuma_run_profiled)",
    }
    if not shared:
        line["roofline"] = {
            "bound": "hbm",
            "achieved": round(equivalent, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(equivalent / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "definition": (f"SURVEY 8d step roofline: scenario-epochs/s per GPU x BYTES(V,M) = {contract:,.0f} B "
                           "(read W, B, S; write B, Dn, C, I) / 8 TB/s; traffic = rocprofv3 FETCH_SIZE + "
                           f"WRITE_SIZE bytes of one step ({os.path.relpath(TRAFFIC_JSON, ROOT)})"),
            "contract_bytes_per_step": contract * units,
            "kernel": kernel,
        }
    else:
        # one shared input trajectory: the sweep scan re-reads W from the
        # caches and is bound by VALU issue, not HBM: the
        # roofline is the dominant kernel's VALU issue rate — its committed
        # SQ_INSTS_VALU per launch (SQ pass of this exact workload) over its
        # live HIP-event time — against the issue peak (1024 SIMDs, a wave64
        # VALU instruction every 2 cycles at 2.4 GHz, MI355X_MICROARCH.md).
        # The PMC bytes beyond L2 are reported apart; they are not an HBM
        # fraction (Infinity-Cache hits count as fetched).
        classes = consensus_classes(params)
        step_s = elapsed / args.steps
        sq = load_sq(key)
        valu = None if sq is None or dom_kernel not in sq else sq[dom_kernel]
        ach = None if valu is None else valu["SQ_INSTS_VALU"] / (dom_ms * 1e-3) / 1e9
        line["roofline"] = {
            "bound": "valu",
            "achieved": None if ach is None else round(ach, 2),
            "peak": VALU_PEAK_GINST,
            "unit": "G VALU wave-instructions/s",
            "frac": None if ach is None else round(ach / VALU_PEAK_GINST, 4),
            "traffic": None if pmc is None or dom_kernel not in pmc else round(pmc[dom_kernel] * units / launches),
            "definition": (f"{dom_kernel}: SQ_INSTS_VALU per launch ({os.path.relpath(SQ_JSON, ROOT)}, "
                           f"build {None if valu is None else valu.get('build_id')}) / its HIP-event launch time; "
                           f"peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction; traffic = its "
                           "rocprofv3 FETCH_SIZE + WRITE_SIZE bytes per launch (beyond L2, Infinity-Cache hits "
                           "included: W is re-read per scenario pair, not an HBM fraction)"),
            "valu_instructions_per_launch": None if valu is None else valu["SQ_INSTS_VALU"],
            "step_bytes_beyond_l2": traffic,
            "step_GBps_beyond_l2": None if traffic is None else round(traffic / step_s / 1e9, 1),
            "equivalent_GBps": round(equivalent, 1),
            "equivalent_definition": (f"scenario-epochs/s per GPU x the per-scenario epoch-step contract "
                                      f"{contract:,.0f} B: a rate, not traffic (every scenario reads one shared "
                                      f"W/S trajectory; row sums once per input epoch, consensus and rank once "
                                      f"per consensus class: {classes} classes of {N})"),
            "kernel": kernel,
        }
        line["config"]["consensus_classes"] = classes
    line["phases"] = phase_info
    return line


def input_seed(config: str, seed: int, rank: int) -> int:
    """Seed of a rank's synthetic inputs: c3 sweeps ONE subnet trajectory on
    every rank (the grid is dealt to the ranks, the subnet is not); c2
    replicas are independent subnets, one per rank."""
    return seed if config == "c3" else seed + 7919 * rank


def bench_engine(args, world: int, rank: int, dist: bool) -> dict:
    """c2 (default) and c3: engine.run over E epochs of N scenarios per GPU."""
    from yuma_simulation._internal import engine, synth
    from yuma_simulation._internal.simulation_utils import resolve_version
    from yuma_simulation._internal.yumas import YumaConfig, YumaParams

    dev = engine.device()
    E, V, M, N = args.epochs, args.validators, args.miners, args.scenarios
    variant, _ = resolve_version(args.version)
    liquid_version = args.version.endswith("liquid alpha on")
    if args.config == "c3":
        # the sweep grid dealt to the ranks: N points per GPU (weak scaling;
        # 8 GPUs x 512 = the whole 4096-point grid)
        from yuma_simulation._internal.sharding import shard_range

        cfgs = [sweep_config(g % 4096) for g in shard_range(N * world, world, rank)]
    else:
        cfgs = [YumaConfig(yuma_params=YumaParams(liquid_alpha=args.liquid or liquid_version))] * N
    params = [engine.make_params(variant, c) for c in cfgs]
    liquid = any(p.liquid_mode != engine.LIQUID_OFF for p in params)
    hist = not args.no_history
    # inputs resident in HBM before timing; the c3 sweep runs every scenario
    # over ONE subnet trajectory (shared W/S, params vary), the
    # same on every rank (the 4096-point grid dealt to the ranks sweeps one
    # subnet); c2 replicas: each rank simulates its own subnet
    shared = args.config == "c3"
    seed = input_seed(args.config, args.seed, rank)
    Nin = 1 if shared else N
    W = engine.synth_weights(seed, E, Nin, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, Nin, V)).to(dev)

    def workload_of(version: str, liq: bool) -> dict:
        if args.config == "c3":
            wl = (f"c3: parameter sweep, {N} scenarios per GPU (of the 4096-point bond_alpha x kappa x "
                  f"liquid x alpha grid) over one shared {V}V x {M}M x {E}-epoch subnet trajectory, {version}")
        else:
            wl = f"c2: single subnet {V}V x {M}M x {E} epochs, {version}" + (" (liquid)" if liq else "")
        return {"workload": wl, "V": V, "M": M, "epochs": E, "scenarios_per_gpu": N, "version": version,
                "bond_history": hist, "launch": "direct" if args.no_graph else "hipGraph replay",
                "parallelism": f"scenario-sharded x{world}" if world > 1 else "single GPU"}

    line = engine_line(args, variant, params, W, S, world, dist, workload_of(args.version, liquid), shared=shared)
    if args.config == "c2" and not args.no_also:
        # SURVEY §7 "Config 2 naming": c2 is quoted for Yuma 3 AND Yuma 4 liquid
        v4 = "Yuma 4 (Rhef+relative bonds) - liquid alpha on"
        p4 = [engine.make_params(4, YumaConfig(yuma_params=YumaParams(liquid_alpha=True)))] * N
        l4 = engine_line(args, 4, p4, W, S, world, dist, workload_of(v4, True))
        line["also"] = {v4: {k: l4[k] for k in ("value", "unit", "ms_per_step", "roofline", "phases", "config")}}
    if rank == 0 and not args.no_cpu_baseline:
        if args.config == "c3":
            line["cpu_baseline"] = cpu_baseline("yuma4" if variant == 4 else "yuma3", W, S, cfgs[:8], 10.0, 1, 1,
                                                "c3: first 8 sweep scenarios")
        else:
            vname = {0: "rust", 1: "yuma1", 2: "yuma2", 3: "yuma3", 4: "yuma4"}[variant]
            line["cpu_baseline"] = cpu_baseline(vname, W, S, cfgs[:1], 10.0, 2, args.cpu_structured_epochs,
                                                f"c2: {args.version}")
    return line


def bench_wide(args, world: int, rank: int, dist: bool) -> dict:
    """c4: one wide subnet, miner columns sharded across the ranks."""
    from yuma_simulation._internal import engine, synth, wide
    from yuma_simulation._internal.simulation_utils import resolve_version
    from yuma_simulation._internal.yumas import YumaConfig

    dev = engine.device()
    E, V, M = args.epochs, args.validators, args.miners
    variant, _ = resolve_version(args.version)
    params = [engine.make_params(variant, YumaConfig())]
    cols = wide.column_ranges(M, world)[rank]
    W = engine.synth_weights(args.seed, E, 1, V, M)[..., cols.start:cols.stop].contiguous()
    torch.cuda.empty_cache()
    S = torch.from_numpy(synth.stakes(args.seed, E, 1, V)).to(dev)
    hist = not args.no_history
    if dist:
        def step():
            return wide.run_wide_distributed(variant, params, W, S, M_total=M, want_hist=hist)
    else:
        # one GPU holds the whole subnet: the unsharded engine (one yuma_run),
        # no shard stages or exchanges
        ws = torch.empty(engine.workspace_bytes(variant, 1, E, V, M, False), dtype=torch.uint8, device=dev)

        def step():
            return engine.run(variant, params, W, S, want_hist=hist, workspace=ws)

    elapsed = timed(step, args.warmup, args.steps, dist, dev)
    value = float(E) * args.steps / elapsed  # one subnet: total work fixed
    per_gpu_bytes = contract_bytes(V, len(cols), variant) * E * args.steps / elapsed / 1e9
    layout = f"miner columns sharded x{world}" if dist else "unsharded, one GPU"
    workload = {"workload": f"c4: wide subnet {V}V x {M}M x {E} epochs, {args.version}, {layout}", "V": V, "M": M, "epochs": E, "scenarios_per_gpu": 1,
                "version": args.version, "bond_history": hist,
                "parallelism": (f"miner-column sharded x{world} (all-gather of per-shard partials)" if dist
                                else "single GPU, unsharded engine")}
    line = base_line(args, world, value, "scenario-epochs/s", elapsed, "strong", workload)
    pmc = load_traffic({k: workload[k] for k in ("V", "M", "epochs", "scenarios_per_gpu", "version",
                                                  "bond_history")}) if world == 1 else None
    line["roofline"] = {"bound": "hbm", "achieved": round(per_gpu_bytes, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": round(per_gpu_bytes / HBM_PEAK_GBPS, 4),
                        "traffic": None if pmc is None else round(sum(pmc.values()) * E),
                        "definition": "SURVEY 8d step roofline per GPU: BYTES(V, M/world) x epochs/s / 8 TB/s "
                                      "(all stages and exchanges inside the wall time)"}
    if not dist:
        # per-phase device time of the same run (HIP events, yuma_run_profiled)
        # and the dominant kernel's roofline, as for c2
        buf = [0.0] * len(engine.PHASES)
        engine.run(variant, params, W, S, want_hist=hist, workspace=ws, phase_ms=buf)
        liquid = any(p.liquid_mode != engine.LIQUID_OFF for p in params)
        phases = {}
        for i, name in enumerate(engine.PHASES):
            kname = kernel_of(name, variant, False, V, M)
            if buf[i] > 0:
                b = phase_bytes(name, V, M, variant, liquid, hist, E) * E
                phases[name] = {"kernel": kname, "ms": round(buf[i], 4),
                                "GBps": round(b / (buf[i] * 1e-3) / 1e9, 1)}
        dom = max(phases, key=lambda k: phases[k]["ms"])
        dk = kernel_of(dom, variant, False, V, M)
        db = phase_bytes(dom, V, M, variant, liquid, hist, E) * E
        line["roofline"]["kernel"] = {
            "name": dk, "launches_per_step": 1, "avg_ms": phases[dom]["ms"], "bytes_per_launch": db,
            "achieved": phases[dom]["GBps"], "frac": round(phases[dom]["GBps"] / HBM_PEAK_GBPS, 4),
            "traffic": None if pmc is None or dk not in pmc else round(pmc[dk] * E),
            "timing": "HIP events on the launch stream around the kernel (yuma_run_profiled)"}
        line["phases"] = phases
    if rank == 0 and not args.no_cpu_baseline and variant in (3, 4):
        Wc = engine.synth_weights(args.seed, 3, 1, V, M)  # the full-width first epochs, for the CPU
        line["cpu_baseline"] = cpu_baseline({3: "yuma3", 4: "yuma4"}[variant], Wc, S, [YumaConfig()], 10.0, 1, 0,
                                            f"c4: {args.version} at {V}x{M}")
        del Wc
    return line


def bench_sheet(args, world: int, rank: int, dist: bool) -> dict:
    """c5: the dividend sheet of all four bond penalties (504 runs)."""
    from yuma_simulation._internal import engine
    from yuma_simulation._internal.cases import cases
    from yuma_simulation._internal.simulation_utils import (
        SHEET_BOND_PENALTIES,
        _sheet_runs,
        generate_total_dividends_tables,
        run_simulations,
        sheet_yuma_versions,
    )
    from yuma_simulation._internal.yumas import SimulationHyperparameters

    dev = engine.device()
    hypers = [SimulationHyperparameters(bond_penalty=b) for b in SHEET_BOND_PENALTIES]
    versions = sheet_yuma_versions()
    runs = [r for h in hypers for r in _sheet_runs(cases, versions, h)]
    units = sum(r.case.num_epochs for r in runs)
    if dist:
        mine = runs[rank::world]

        def step():
            return run_simulations(mine, want_bonds=False, want_incentives=False)
    else:
        def step():
            return generate_total_dividends_tables(cases, versions, hypers)

    elapsed = timed(step, args.warmup, args.steps, dist, dev)
    value = units * args.steps / elapsed
    workload = {"workload": f"c5: dividend sheet, {len(runs)} runs (4 bond penalties x {len(cases)} cases x "
                            f"{len(versions)} versions), {units} scenario-epochs", "runs": len(runs),
                "scenario_epochs": units, "parallelism": f"runs sharded x{world}" if world > 1 else "single GPU"}
    line = base_line(args, world, value, "scenario-epochs/s", elapsed, "strong", workload)
    line["data"] = "the reference's built-in cases (cases.py)"
    line["roofline"] = {"bound": "latency", "kernel": "whole sheet (3x2 matrices: launch/host bound)",
                        "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None}
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = sheet_cpu_baseline(len(runs), units)
    return line


def _sheet_worker_init():
    import torch as _t

    _t.set_num_threads(1)
    _sheet_chunk([0])  # warm: imports, case construction


def _sheet_chunk(idx: list) -> float:
    """Worker: run_simulation (oracle/torch_cpu.py, bit-identical to the
    reference's dividend lists) for the sheet runs `idx`; returns seconds."""
    from oracle import torch_cpu as tc
    from yuma_simulation._internal.cases import cases
    from yuma_simulation._internal.simulation_utils import SHEET_BOND_PENALTIES, _sheet_runs, sheet_yuma_versions
    from yuma_simulation._internal.yumas import SimulationHyperparameters

    runs = [r for b in SHEET_BOND_PENALTIES
            for r in _sheet_runs(cases, sheet_yuma_versions(), SimulationHyperparameters(bond_penalty=b))]
    t0 = time.perf_counter()
    for i in idx:
        r = runs[i]
        c = r.case
        tc.run_simulation(r.yuma_version, c.weights_epochs, c.stakes_epochs, r.yuma_config, c.num_epochs,
                          c.validators, c.reset_bonds_epoch, c.reset_bonds_index)
    return time.perf_counter() - t0


def sheet_cpu_baseline(n_runs: int, units: int) -> dict:
    """c5 CPU baseline: the reference's run_simulation restated in CPU torch
    (oracle/torch_cpu.run_simulation) over all sheet runs, dealt round-robin to
    one single-threaded worker process per CPU of this process's share (3 x 2
    matrices: intra-op threads cannot help, independent runs can)."""
    import multiprocessing as mp

    host = host_cpu()
    k = max(1, host["threads"])
    chunks = [list(range(i, n_runs, k)) for i in range(k)]
    ctx = mp.get_context("spawn")  # the parent holds a GPU context: never fork it
    with ctx.Pool(k, initializer=_sheet_worker_init) as pool:
        pool.map(_sheet_chunk, [[0]] * k)  # every worker started and warm
        t0 = time.perf_counter()
        busy = pool.map(_sheet_chunk, chunks)
        dt = time.perf_counter() - t0
    return {"value": round(units / dt, 1), "unit": "scenario-epochs/s", "cores": k, "kind": "port",
            "sample": (f"all {n_runs} sheet runs ({units} scenario-epochs): oracle/torch_cpu.run_simulation "
                       f"(bit-identical to the reference's dividend lists, tests/test_oracle_golden.py), dealt to "
                       f"{k} single-threaded worker processes ({host['share']}); {dt:.2f} s wall, "
                       f"{max(busy):.2f} s on the busiest worker, on {host['model']}"),
            "host": host}


DEFAULTS = {  # per config: epochs, validators, miners, scenarios per GPU, version, history
    "c2": (1000, 256, 4096, 1, "Yuma 3 (Rhef)", True),
    "c3": (32, 256, 4096, 512, "Yuma 4 (Rhef+relative bonds)", False),
    "c4": (100, 256, 65536, 1, "Yuma 3 (Rhef)", False),
    "c5": (40, 3, 2, 1, "", False),
}


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(DEFAULTS), default="c2",
                    help="BASELINE.json workload (c2 is the headline metric)")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--validators", type=int, default=None)
    ap.add_argument("--miners", type=int, default=None)
    ap.add_argument("--scenarios", type=int, default=None, help="scenarios per GPU")
    ap.add_argument("--version", default=None)
    ap.add_argument("--liquid", action="store_true")
    ap.add_argument("--no-history", action="store_true", help="do not write every epoch's bond state")
    ap.add_argument("--chunk", type=int, default=0, help="epochs per phase-1 batch (0 = engine default)")
    ap.add_argument("--no-graph", action="store_true",
                    help="c2/c3: launch each step directly instead of replaying a captured hipGraph")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=None)
    ap.add_argument("--cpu-structured-epochs", type=int, default=10,
                    help="c2: timed epochs of the reference-structured CPU baseline (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-also", action="store_true", help="c2: skip the Yuma 4 liquid companion line")
    ap.add_argument("--profile-reps", type=int, default=3)
    args = ap.parse_args()
    E, V, M, N, version, hist = DEFAULTS[args.config]
    args.epochs = args.epochs or E
    args.validators = args.validators or V
    args.miners = args.miners or M
    args.scenarios = args.scenarios or N
    args.version = args.version or version
    if not hist:
        args.no_history = True
    if args.seed is None:
        args.seed = {"c3": 0x5EED0003, "c4": 0x5EED0004}.get(args.config, 0x5EED0002)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: re-launch under torch.distributed.run before
        # anything here has touched a GPU, and exit with its status
        import socket
        import subprocess

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        if BACKEND == "gloo":
            # rehearsal of the N-rank path on a box with fewer GPUs: ranks share
            # the card(s), collectives go through host memory
            torch.cuda.set_device(local % torch.cuda.device_count())
            tdist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    run = {"c2": bench_engine, "c3": bench_engine, "c4": bench_wide, "c5": bench_sheet}[args.config]
    line = run(args, world, rank, dist)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        # rank 0 may still be timing its CPU baseline: leave together
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
