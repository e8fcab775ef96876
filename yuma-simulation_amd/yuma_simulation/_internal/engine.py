"""ctypes binding of libyuma_hip.so (include/yuma_hip.h) — the only compute path.

The product never falls back to CPU: if the HIP library or a GPU is missing,
every compute entry point raises ``EngineUnavailable``. Tensors are handed over
as raw device pointers; the engine is stream-ordered on torch's current stream
and allocates nothing (the workspace is a torch uint8 tensor).

Parameter marshalling mirrors how the reference's torch ops round Python
scalars (yumas.py:7-45 configs, used at :186-262 and copies):
  * a Python float meeting an fp32 tensor is rounded to fp32 first;
  * ``1 - x`` of two Python floats is computed in double, then rounded;
  * the bisection trip count is the reference's own loop evaluated in double.
"""

from __future__ import annotations

import ctypes
import math
import numbers
import operator
import os
import threading
from dataclasses import dataclass

import numpy as np
import torch

LIB_NAME = "libyuma_hip.so"
_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.environ.get("YUMA_HIP_LIB", os.path.join(_PKG_ROOT, "lib", LIB_NAME))

VARIANT_RUST, VARIANT_YUMA1, VARIANT_YUMA2, VARIANT_YUMA3, VARIANT_YUMA4 = range(5)
PHASES = ("rowsum", "consensus", "quantise", "rank", "incentive", "bonds", "finalize")
FLAG_NO_HIST = 1  # yuma_params_t.flags: plain bisection instead of the histogram finish
FLAG_RESET_ALL_COLUMNS = 2  # the reset zeroes every column (reset_bonds_index None)
RESET_NONE, RESET_ALWAYS, RESET_IF_ZERO_CONSENSUS = range(3)
RUN_SHARED_INPUTS = 1  # yuma_run_ex flags
LIQUID_OFF, LIQUID_QUANTILE, LIQUID_CONST_AB = range(3)
OVR_HIGH, OVR_LOW, OVR_FORCE_Q99 = 1, 2, 4

EXPORTED_SYMBOLS = (
    "yuma_workspace_bytes",
    "yuma_run",
    "yuma_run_profiled",
    "yuma_run_ex",
    "yuma_epoch",
    "yuma_synth_weights",
    "yuma_shard_stage",
    "yuma_graph_create",
    "yuma_graph_create_ex",
    "yuma_graph_launch",
    "yuma_graph_nodes",
    "yuma_graph_destroy",
    "yuma_last_error",
    "yuma_version",
    "yuma_build_id",
)


class EngineUnavailable(RuntimeError):
    """The HIP engine cannot run here (library not built or no GPU)."""


class EngineError(RuntimeError):
    """The engine rejected a call (bad sizes, workspace, launch failure)."""


MAX_VALIDATORS = 1 << 20  # include/yuma_hip.h YUMA_MAX_VALIDATORS
REG_VALIDATORS = 1024  # YUMA_REG_VALIDATORS: above it the engine streams each miner column
MAX_BISECT_ITERS = 30  # consensus_precision <= 2**30: the search grid k / 2**iters in int32


def check_limits(V: int, M: int) -> None:
    """The engine's size limits, checked before anything touches a GPU. The
    reference (yumas.py:195-209) has none; real subnets stay far inside them
    (DESIGN.md §3 'Limits')."""
    if V > MAX_VALIDATORS:
        raise EngineError(f"{V} validators exceed the engine's limit of {MAX_VALIDATORS} per subnet "
                          "(YUMA_MAX_VALIDATORS)")
    if M > (1 << 20) * 64:
        raise EngineError(f"{M} miners exceed the engine's limit of {(1 << 20) * 64} (2^20 tiles of 64)")


class YumaParamsC(ctypes.Structure):
    _fields_ = [
        ("variant", ctypes.c_int32),
        ("bisect_iters", ctypes.c_int32),
        ("liquid_mode", ctypes.c_int32),
        ("override_flags", ctypes.c_int32),
        ("reset_mode", ctypes.c_int32),
        ("reset_epoch", ctypes.c_int32),
        ("reset_index", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("kappa", ctypes.c_float),
        ("bond_penalty", ctypes.c_float),
        ("one_minus_bond_penalty", ctypes.c_float),
        ("bond_alpha", ctypes.c_float),
        ("one_minus_bond_alpha", ctypes.c_float),
        ("alpha_low", ctypes.c_float),
        ("alpha_high", ctypes.c_float),
        ("capacity_alpha", ctypes.c_float),
        ("decay_keep", ctypes.c_float),
        ("maxint", ctypes.c_float),
        ("const_a", ctypes.c_float),
        ("const_b", ctypes.c_float),
        ("ln_num", ctypes.c_double),
        ("ln_low", ctypes.c_double),
        ("override_high", ctypes.c_double),
        ("override_low", ctypes.c_double),
        ("reserved1", ctypes.c_double * 2),
    ]


assert ctypes.sizeof(YumaParamsC) == 128, ctypes.sizeof(YumaParamsC)

OUTPUT_FIELDS = (
    "Dn", "D", "C", "I", "R", "P", "T", "Tv", "Sn", "bond_alpha", "alpha_ab",
    "Wn", "Wc", "Wb", "B_inst", "B_hist", "B_final",
)


class YumaOutputsC(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in OUTPUT_FIELDS]


SHARD_IO_FIELDS = ("rowsum_part", "rowsum", "csum_part", "csum_part_d", "csum", "csum_d",
                   "levels", "rsum_part", "rsum", "levels_all", "dsum_part", "dsum", "tv_part", "tv")


class YumaShardIOC(ctypes.Structure):
    """yuma_shard_io_t (include/yuma_hip.h): two ints, then device pointers."""
    _fields_ = [("M_total", ctypes.c_int), ("col0", ctypes.c_int)] + [
        (name, ctypes.c_void_p) for name in SHARD_IO_FIELDS]


_lock = threading.Lock()
_lib = None


def load_library(path: str | None = None):
    """Load (once) and type the C-ABI library. Raises EngineUnavailable."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("YUMA_LIB") or LIB_PATH  # YUMA_LIB: A/B of two builds (tools/ab_lib.sh)
        if not os.path.exists(p):
            raise EngineUnavailable(
                f"{LIB_NAME} not found at {p}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        try:
            lib = ctypes.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the ROCm runtime
            raise EngineUnavailable(f"cannot load {p}: {e}") from e
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        lib.yuma_workspace_bytes.argtypes = [i32, i32, i32, i32, i32, i32]
        lib.yuma_workspace_bytes.restype = sz
        lib.yuma_run.argtypes = [i32, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, sz, i32, vp]
        lib.yuma_run.restype = i32
        lib.yuma_run_profiled.argtypes = lib.yuma_run.argtypes + [ctypes.POINTER(ctypes.c_float)]
        lib.yuma_run_profiled.restype = i32
        lib.yuma_run_ex.argtypes = lib.yuma_run.argtypes[:-1] + [i32, vp, ctypes.POINTER(ctypes.c_float)]
        lib.yuma_run_ex.restype = i32
        lib.yuma_epoch.argtypes = [i32, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, sz, vp]
        lib.yuma_epoch.restype = i32
        lib.yuma_shard_stage.argtypes = [i32, i32, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp,
                                         vp, sz, vp]
        lib.yuma_shard_stage.restype = i32
        lib.yuma_synth_weights.argtypes = [ctypes.c_uint64, i32, i32, i32, i32, i32, vp, vp]
        lib.yuma_synth_weights.restype = i32
        lib.yuma_graph_create.argtypes = [ctypes.POINTER(vp), i32, vp, i32, i32, i32, i32, vp, vp,
                                          vp, vp, vp, vp, sz, i32]
        lib.yuma_graph_create.restype = i32
        lib.yuma_graph_create_ex.argtypes = lib.yuma_graph_create.argtypes + [i32]
        lib.yuma_graph_create_ex.restype = i32
        lib.yuma_graph_launch.argtypes = [vp, vp]
        lib.yuma_graph_launch.restype = i32
        lib.yuma_graph_nodes.argtypes = [vp]
        lib.yuma_graph_nodes.restype = i32
        lib.yuma_graph_destroy.argtypes = [vp]
        lib.yuma_graph_destroy.restype = i32
        lib.yuma_last_error.argtypes = []
        lib.yuma_last_error.restype = ctypes.c_char_p
        lib.yuma_version.argtypes = []
        lib.yuma_version.restype = ctypes.c_char_p
        if hasattr(lib, "yuma_build_id"):  # (A/B libraries of older sources lack it)
            lib.yuma_build_id.argtypes = []
            lib.yuma_build_id.restype = ctypes.c_char_p
        _lib = lib
        return lib


def device() -> torch.device:
    """The GPU the engine runs on; raises EngineUnavailable without one."""
    if not torch.cuda.is_available():
        raise EngineUnavailable("the Yuma HIP engine needs a ROCm GPU (torch.cuda.is_available() is False)")
    load_library()
    return torch.device("cuda", torch.cuda.current_device())


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().yuma_last_error().decode(errors="replace")
        raise EngineError(f"{what} failed ({rc}): {msg}")


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


# ---------------------------------------------------------------------------
# parameter marshalling
# ---------------------------------------------------------------------------
def bisect_iterations(consensus_precision) -> int:
    """Trip count of `while (c_high - c_low) > 1 / precision` (yumas.py:201):
    the interval halves exactly every iteration, independent of the data."""
    threshold = 1 / consensus_precision
    hi, lo, n = 1.0, 0.0, 0
    while (hi - lo) > threshold:
        hi = (hi + lo) / 2.0
        n += 1
        if n > 4096:  # pragma: no cover - nonsensical precision
            raise ValueError("consensus_precision too large")
    return n


def f32(x) -> float:
    return float(np.float32(x))


def make_params(variant: int, config, *, maxint: int = 2**64 - 1, reset_mode: int = RESET_NONE,
                reset_epoch: int | None = None, reset_index: int | None = None,
                n_miners: int | None = None, n_epochs: int | None = None) -> YumaParamsC:
    """Flatten a YumaConfig (yumas.py:29-45) into the engine's POD record."""
    p = YumaParamsC()
    p.variant = variant
    p.bisect_iters = bisect_iterations(config.consensus_precision)
    if p.bisect_iters > MAX_BISECT_ITERS:
        raise EngineError(f"consensus_precision {config.consensus_precision} needs {p.bisect_iters} bisection "
                          f"steps; the engine supports at most {MAX_BISECT_ITERS} (consensus_precision <= 2**30)")
    p.kappa = f32(config.kappa)
    p.bond_penalty = f32(config.bond_penalty)
    p.one_minus_bond_penalty = f32(1 - config.bond_penalty)
    p.bond_alpha = f32(config.bond_alpha)
    p.one_minus_bond_alpha = f32(1 - config.bond_alpha)
    p.alpha_low = f32(config.alpha_low)
    p.alpha_high = f32(config.alpha_high)
    p.capacity_alpha = f32(config.capacity_alpha)
    p.decay_keep = f32(1 - config.decay_rate)
    p.maxint = f32(float(maxint))
    p.const_a = p.const_b = float("nan")
    p.override_high = p.override_low = float("nan")
    p.liquid_mode = LIQUID_OFF
    uses_liquid = variant in (VARIANT_RUST, VARIANT_YUMA1, VARIANT_YUMA2, VARIANT_YUMA4)
    if config.liquid_alpha and uses_liquid:
        # the reference evaluates these when it reaches them (yumas.py:248-251);
        # math.log raises ValueError for alpha outside (0, 1) exactly as there
        ln_high = math.log(1 / config.alpha_high - 1)
        ln_low = math.log(1 / config.alpha_low - 1)
        p.ln_num = ln_high - ln_low
        p.ln_low = ln_low
        hi_o, lo_o = config.override_consensus_high, config.override_consensus_low
        flags = 0
        if hi_o is not None:
            flags |= OVR_HIGH
            p.override_high = float(hi_o)
        if lo_o is not None:
            flags |= OVR_LOW
            p.override_low = float(lo_o)
        p.liquid_mode = LIQUID_QUANTILE
        if hi_o is not None and lo_o is not None:
            if hi_o == lo_o:  # python comparison, then consensus_high = quantile(.99)
                flags |= OVR_FORCE_Q99
            else:  # pure-python a, b (doubles), rounded when they meet C
                a = (ln_high - ln_low) / (lo_o - hi_o)
                b = ln_low + a * lo_o
                p.const_a, p.const_b = f32(a), f32(b)
                p.liquid_mode = LIQUID_CONST_AB
        p.override_flags = flags
    _pack_reset(p, reset_mode, reset_epoch, reset_index, n_miners, n_epochs)
    return p


_PARAMS_CACHE: dict = {}
_CONFIG_FIELDS = ("consensus_precision", "kappa", "bond_penalty", "bond_alpha", "alpha_low", "alpha_high",
                  "capacity_alpha", "decay_rate", "liquid_alpha", "override_consensus_high",
                  "override_consensus_low")


def config_key(config) -> tuple:
    """The values make_params reads from a config (repr: -0.0 and 0.0 differ)."""
    return tuple(repr(getattr(config, f)) for f in _CONFIG_FIELDS)


def make_params_cached(variant: int, config, *, reset_mode: int = RESET_NONE, reset_epoch=None,
                       reset_index=None, n_miners: int | None = None, n_epochs: int | None = None,
                       ckey: tuple | None = None) -> YumaParamsC:
    """make_params memoised on every value it reads (the sheet builds 504
    records from 36 distinct configurations). Plain int / None reset fields
    only; anything else (a tensor-valued reset epoch) is built fresh. The
    record is shared: callers copy it into the device tensor, never mutate it.
    ckey: config_key(config), when the caller already has it."""
    if not all(x is None or type(x) is int for x in (reset_epoch, reset_index)):
        return make_params(variant, config, reset_mode=reset_mode, reset_epoch=reset_epoch,
                           reset_index=reset_index, n_miners=n_miners, n_epochs=n_epochs)
    key = (variant, reset_mode, reset_epoch, reset_index, n_miners, n_epochs,
           config_key(config) if ckey is None else ckey)
    p = _PARAMS_CACHE.get(key)
    if p is None:
        p = make_params(variant, config, reset_mode=reset_mode, reset_epoch=reset_epoch,
                        reset_index=reset_index, n_miners=n_miners, n_epochs=n_epochs)
        if len(_PARAMS_CACHE) > 65536:
            _PARAMS_CACHE.clear()
        _PARAMS_CACHE[key] = p
    return p


class _NoTruthValue(Exception):
    """reset_bonds_epoch is a tensor / array whose `epoch == e` has no truth value."""

    def __init__(self, value):
        super().__init__()
        self.value = value


def _reset_epoch_value(reset_epoch) -> int | None:
    """The int epoch e at which the reference's `epoch == case.reset_bonds_epoch`
    (simulation_utils.py:63,70,81; epoch an int from range()) holds, or None
    when it never does: ints and bools (True == 1) as themselves, a float only
    when integral (20.0 == 20, 20.5 never), a one-element tensor or array as
    its element (`epoch == tensor(20)` is a truthy tensor), anything else
    never. Tensors and arrays of any other size have no truth value: the
    caller raises the reference's own error when the statement is reached."""
    if isinstance(reset_epoch, (torch.Tensor, np.ndarray)):
        n = reset_epoch.numel() if isinstance(reset_epoch, torch.Tensor) else reset_epoch.size
        if n != 1:
            raise _NoTruthValue(reset_epoch)
        return _reset_epoch_value(reset_epoch.item())
    if isinstance(reset_epoch, (bool, np.bool_, numbers.Integral)):
        return int(reset_epoch)
    if isinstance(reset_epoch, numbers.Real):
        f = float(reset_epoch)
        return int(f) if f.is_integer() else None
    return None


def _pack_reset(p: YumaParamsC, reset_mode: int, reset_epoch, reset_index, n_miners, n_epochs) -> None:
    """The bond reset of run_simulation (simulation_utils.py:62-88) with the
    reference's Python indexing: `B_state[:, idx] = 0.0` and
    `server_consensus_weight[idx] == 0.0`, evaluated only at
    `epoch == reset_bonds_epoch` once B_state exists (epoch >= 1).

    - reset_epoch None or a non-integral number: never equal, no reset;
      epochs below 1 are never reached (B_state is None at epoch 0);
    - negative index: counts from the end (idx % M);
    - index None or True: `B_state[:, None]` / `B_state[:, True]` zeroes every
      column (Yuma 3.1); Yuma 3.2/4 also evaluate `scw[idx] == 0.0`, a [1, M]
      tensor whose truth value raises RuntimeError for M > 1 (for M == 1 it is
      column 0);
    - index False: `B_state[:, False]` selects nothing (Yuma 3.1: no reset);
      Yuma 3.2/4's `scw[False] == 0.0` is an empty tensor whose truth value
      raises RuntimeError;
    - index outside [-M, M): IndexError.
    The errors are raised only when the reference would reach the statement
    (reset_epoch in [1, n_epochs)). n_miners is needed for anything but a
    plain in-range non-negative index."""
    p.reset_mode = RESET_NONE
    p.reset_epoch = -1
    p.reset_index = 0
    if reset_mode == RESET_NONE or reset_epoch is None:
        return
    try:
        epoch = _reset_epoch_value(reset_epoch)
    except _NoTruthValue as e:
        if n_epochs is None or n_epochs >= 2:  # reached at epoch 1: the reference's own error
            bool(1 == e.value)
        return
    if epoch is None or epoch < 1 or (n_epochs is not None and epoch >= n_epochs):
        return  # the statement never runs
    if not -2**31 <= epoch < 2**31:
        return  # beyond any int32 epoch count: never equal
    if isinstance(reset_index, (bool, np.bool_)) and not reset_index:
        if reset_mode == RESET_IF_ZERO_CONSENSUS:
            raise RuntimeError("Boolean value of Tensor with no values is ambiguous "
                               "(server_consensus_weight[False] == 0.0, simulation_utils.py:72,83)")
        return  # B_state[:, False] = 0.0 touches nothing
    if reset_index is None or isinstance(reset_index, (bool, np.bool_)):
        if n_miners is None:
            raise ValueError("a reset with reset_bonds_index None needs n_miners")
        if reset_mode == RESET_IF_ZERO_CONSENSUS and n_miners > 1:
            raise RuntimeError("Boolean value of Tensor with more than one value is ambiguous "
                               f"(server_consensus_weight[{reset_index}] == 0.0, simulation_utils.py:72,83)")
        if reset_mode == RESET_ALWAYS:
            p.flags |= FLAG_RESET_ALL_COLUMNS
            idx = 0
        else:
            idx = 0  # M == 1: scw[None] is the single column
    else:
        idx = operator.index(reset_index)
        if n_miners is not None:
            if not -n_miners <= idx < n_miners:
                raise IndexError(f"index {idx} is out of bounds for dimension 1 with size {n_miners}")
            idx %= n_miners
        elif idx < 0:
            raise ValueError("a negative reset_bonds_index needs n_miners to resolve")
    p.reset_mode = reset_mode
    p.reset_epoch = epoch
    p.reset_index = idx


def params_tensor(params: list[YumaParamsC], dev: torch.device) -> torch.Tensor:
    raw = b"".join(bytes(p) for p in params)
    host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    return host.to(dev)


# ---------------------------------------------------------------------------
# engine calls
# ---------------------------------------------------------------------------
@dataclass
class RunResult:
    Dn: torch.Tensor                  # [E, N, V]
    C: torch.Tensor                   # [E, N, M]
    I: torch.Tensor                   # [E, N, M]
    B_final: torch.Tensor             # [N, V, M]
    B_hist: torch.Tensor | None       # [E, N, V, M]
    extra: dict


def _as_dev(x: torch.Tensor, dev) -> torch.Tensor:
    return x.to(device=dev, dtype=torch.float32).contiguous()


def workspace_bytes(variant: int, N: int, E: int, V: int, M: int, full: bool) -> int:
    return int(load_library().yuma_workspace_bytes(variant, N, E, V, M, 1 if full else 0))


def run(variant: int, params: list[YumaParamsC], W: torch.Tensor, S: torch.Tensor,
        B_init: torch.Tensor | None = None, Wprev_init: torch.Tensor | None = None, *,
        want_hist: bool = False, want: tuple[str, ...] = (), chunk_epochs: int = 0,
        workspace: torch.Tensor | None = None, out: dict | None = None,
        phase_ms: list | None = None, capture: list | None = None,
        single_call: bool = False, shared_inputs: bool = False) -> RunResult:
    """E epochs of N scenarios. W [E,N,V,M], S [E,N,V] (raw); optional
    B_init [N,V,M] and (Yuma2) normalised Wprev_init [N,V,M].
    single_call: E == 1 through yuma_epoch (one call of a Yuma* variant,
    yumas.py:61/175/285/399/494) instead of yuma_run.
    shared_inputs: W [E,1,V,M] and S [E,1,V] are one trajectory that every
    scenario (one per params record) reads — a parameter sweep over one subnet
    (yuma_run_ex, YUMA_RUN_SHARED_INPUTS); results equal a run on W and S
    replicated per scenario."""
    E, Nw, V, M = W.shape
    check_limits(V, M)
    dev = device()
    lib = load_library()
    if S.shape != (E, Nw, V):
        raise ValueError(f"S shape {tuple(S.shape)} does not match W {tuple(W.shape)}")
    if shared_inputs:
        if Nw != 1:
            raise ValueError("shared_inputs takes W [E,1,V,M] and S [E,1,V]")
        N = len(params)
        if single_call:
            raise ValueError("single_call does not take shared inputs")
    else:
        N = Nw
        if len(params) != N:
            raise ValueError("one parameter record per scenario is required")
    W = _as_dev(W, dev)
    S = _as_dev(S, dev)
    B_init = None if B_init is None else _as_dev(B_init, dev)
    Wprev_init = None if Wprev_init is None else _as_dev(Wprev_init, dev)
    prm = params_tensor(params, dev)
    o = {} if out is None else dict(out)

    def need(name, shape):
        if name not in o or o[name] is None:
            o[name] = torch.empty(shape, dtype=torch.float32, device=dev)

    need("Dn", (E, N, V))
    need("C", (E, N, M))
    need("I", (E, N, M))
    need("B_final", (N, V, M))
    if want_hist:
        need("B_hist", (E, N, V, M))
    shapes = {
        "D": (E, N, V), "R": (E, N, M), "P": (E, N, M), "T": (E, N, M), "Tv": (E, N, V),
        "Sn": (E, N, V), "bond_alpha": (E, N, M), "alpha_ab": (E, N, 2),
        "Wn": (E, N, V, M), "Wc": (E, N, V, M), "Wb": (E, N, V, M), "B_inst": (E, N, V, M),
    }
    for name in want:
        need(name, shapes[name])
    if "T" in o and "P" not in o:
        need("P", shapes["P"])
    full = o.get("Tv") is not None
    nbytes = workspace_bytes(variant, N, E, V, M, full)
    if workspace is None or workspace.numel() < nbytes:
        workspace = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    outs = YumaOutputsC(**{k: _ptr(o.get(k)) for k in OUTPUT_FIELDS})
    stream = torch.cuda.current_stream(dev).cuda_stream
    args = (variant, prm.data_ptr(), N, E, V, M, W.data_ptr(), S.data_ptr(),
            _ptr(B_init), _ptr(Wprev_init), ctypes.addressof(outs),
            workspace.data_ptr(), workspace.numel(), int(chunk_epochs), stream)
    if single_call:  # one Yuma* call per slice: the yuma_epoch entry point
        if E != 1 or capture is not None or phase_ms is not None:
            raise ValueError("single_call is one epoch, launched directly")
        _check(lib.yuma_epoch(variant, prm.data_ptr(), N, V, M, W.data_ptr(), _ptr(Wprev_init),
                              S.data_ptr(), _ptr(B_init), ctypes.addressof(outs), workspace.data_ptr(),
                              workspace.numel(), stream), "yuma_epoch")
    elif capture is not None:  # RunGraph: capture instead of launching
        h = ctypes.c_void_p()
        torch.cuda.synchronize(dev)
        if shared_inputs:
            _check(lib.yuma_graph_create_ex(ctypes.byref(h), *args[:-1], RUN_SHARED_INPUTS),
                   "yuma_graph_create_ex")
        else:
            _check(lib.yuma_graph_create(ctypes.byref(h), *args[:-1]), "yuma_graph_create")
        capture.append(h)
    elif shared_inputs:
        buf = None if phase_ms is None else (ctypes.c_float * len(PHASES))()
        _check(lib.yuma_run_ex(*args[:-1], RUN_SHARED_INPUTS, stream, buf), "yuma_run_ex")
        if phase_ms is not None:
            phase_ms[:] = list(buf)
    elif phase_ms is None:
        _check(lib.yuma_run(*args), "yuma_run")
    else:  # bench-only: per-phase device time from HIP events (blocks)
        buf = (ctypes.c_float * len(PHASES))()
        _check(lib.yuma_run_profiled(*args, buf), "yuma_run_profiled")
        phase_ms[:] = list(buf)
    keep = {k: v for k, v in o.items() if k not in ("Dn", "C", "I", "B_final", "B_hist")}
    # keep inputs alive until the stream has consumed them
    keep["_inputs"] = (W, S, B_init, Wprev_init, prm, workspace)
    return RunResult(o["Dn"], o["C"], o["I"], o["B_final"], o.get("B_hist"), keep)


class RunGraph:
    """A whole `run` captured once into a HIP graph (yuma_graph_create) and
    replayed with one launch per call: the E-epoch loop of run_simulation
    (simulation_utils.py:52-110) with no host work between phases or epochs.
    Inputs and outputs are the buffers of the capture (`result`); refill the
    inputs in place between replays."""

    def __init__(self, variant: int, params: list[YumaParamsC], W: torch.Tensor, S: torch.Tensor,
                 B_init: torch.Tensor | None = None, Wprev_init: torch.Tensor | None = None, **kw):
        self._lib = load_library()
        h: list = []
        self.result = run(variant, params, W, S, B_init, Wprev_init, capture=h, **kw)
        self._h = h[0]

    def launch(self) -> RunResult:
        stream = torch.cuda.current_stream(device()).cuda_stream
        _check(self._lib.yuma_graph_launch(self._h, stream), "yuma_graph_launch")
        return self.result

    def nodes(self) -> int:
        return int(self._lib.yuma_graph_nodes(self._h))

    def close(self) -> None:
        if self._h is not None:
            self._lib.yuma_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_stage(stage: int, variant: int, prm: torch.Tensor, W: torch.Tensor, S: torch.Tensor,
                B_init: torch.Tensor | None, Wprev_init: torch.Tensor | None, *, M_total: int,
                col0: int, io: dict, out: dict, workspace: torch.Tensor) -> None:
    """One stage of a miner-column-sharded run (yuma_shard_stage). W [E,N,V,M]
    holds this shard's columns; `io` maps SHARD_IO_FIELDS to device tensors;
    `out` maps OUTPUT_FIELDS to device tensors (local columns)."""
    lib = load_library()
    E, N, V, M = W.shape
    for k in io:
        if k not in SHARD_IO_FIELDS:
            raise KeyError(f"unknown shard io field {k}")
    cio = YumaShardIOC(M_total=int(M_total), col0=int(col0),
                       **{k: _ptr(io.get(k)) for k in SHARD_IO_FIELDS})
    outs = YumaOutputsC(**{k: _ptr(out.get(k)) for k in OUTPUT_FIELDS})
    stream = torch.cuda.current_stream(W.device).cuda_stream
    _check(lib.yuma_shard_stage(stage, variant, prm.data_ptr(), N, E, V, M, W.data_ptr(),
                                S.data_ptr(), _ptr(B_init), _ptr(Wprev_init),
                                ctypes.addressof(cio), ctypes.addressof(outs),
                                workspace.data_ptr(), workspace.numel(), stream),
           f"yuma_shard_stage({stage})")


def synth_weights(seed: int, E: int, N: int, V: int, M: int, t0: int = 0,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Device twin of synth.weights (bit-identical)."""
    dev = device()
    if out is None:
        out = torch.empty((E, N, V, M), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    _check(load_library().yuma_synth_weights(int(seed) & 0xFFFFFFFFFFFFFFFF, E, N, V, M, t0,
                                             out.data_ptr(), stream), "yuma_synth_weights")
    return out


def version() -> str:
    return load_library().yuma_version().decode()


def build_id() -> str:
    """The library's source identity (yuma_build_id: "src-" + SHA-256 prefix of
    the engine source and header it was built from)."""
    lib = load_library()
    return lib.yuma_build_id().decode() if hasattr(lib, "yuma_build_id") else "unstamped"

