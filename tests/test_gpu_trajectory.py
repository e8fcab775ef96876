"""Bench-length trajectories against an independently run oracle (VERDICT r5
weak 1 / next item 3).

test_gpu_long.py pins the 1000-epoch c2 graph to the engine's own chunked run
and resumes the oracle from the engine's bond state for the last two epochs.
Here the oracle runs the whole trajectory itself, from B = None, so rounding
drift over the bench length is shown, not inferred:

  * c2 (the timed step): 256 x 4096 x 1000 epochs of Yuma 3 on the §8d inputs,
    the captured hipGraph vs the oracle's epoch loop (numpy on the box's CPU,
    streamed one epoch at a time). C exact at every epoch, Dn / I within 1e-5
    at every epoch, B_hist BITWISE at epochs 0, 99, ..., 999 (Yuma 3's update
    does not read C and is element-wise in the reference's op order,
    yumas.py:452-472; W / row sum and S / sum(S) are exact-friendly);
  * every sheet version (simulation_utils.py:52-93 dispatch), 320 epochs from
    scratch at 64 x 1024 (the per-tile scans) and 128 x 1024 (the strip scan /
    element-wise column-normalised scans above 64 validators), with resets
    where the version has them: C exact, Dn / I / B within 1e-5 at every epoch.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import yuma_oracle as orc

pytestmark = pytest.mark.gpu

from yuma_simulation._internal import engine, synth  # noqa: E402
from yuma_simulation._internal.simulation_utils import VERSION_TABLE  # noqa: E402
from yuma_simulation._internal.yumas import YumaConfig, YumaParams  # noqa: E402

import bench  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a ROCm GPU"
    engine.load_library()
    yield
    torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_c2_yuma3_1000_epochs_against_oracle_from_scratch():
    """The c2 timed launch (bench.engine_line: RunGraph, Yuma 3, history, one
    chunk) against orc.epoch threaded from B = None for all 1000 epochs."""
    E, V, M = 1000, 256, 4096
    seed = bench.input_seed("c2", 0x5EED0002, 0)
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V)).to(W.device)
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=False))
    g = engine.RunGraph(engine.VARIANT_YUMA3, [engine.make_params(engine.VARIANT_YUMA3, cfg)], W, S,
                        want_hist=True)
    a = g.launch()
    torch.cuda.synchronize()
    C, Dn, I = a.C[:, 0].cpu().numpy(), a.Dn[:, 0].cpu().numpy(), a.I[:, 0].cpu().numpy()
    Sh = S[:, 0].cpu().numpy()
    checkpoints = set(range(0, E, 99)) | {E - 1}
    B = None
    bitwise = 0
    for t in range(E):
        r = orc.epoch("yuma3", W[t, 0].cpu().numpy(), Sh[t], B, cfg)
        B = r["validator_bonds"]
        np.testing.assert_array_equal(C[t], r["server_consensus_weight"], err_msg=f"C[{t}]")
        assert_close(Dn[t], r["validator_reward_normalized"], what=f"Dn[{t}]")
        assert_close(I[t], r["server_incentive"], what=f"I[{t}]")
        if t in checkpoints:
            Bg = a.B_hist[t, 0].cpu().numpy()
            assert np.array_equal(Bg.view(np.uint32), B.view(np.uint32)), (
                f"B[{t}] not bitwise: {int((Bg != B).sum())} elements differ, "
                f"max rel {float(np.max(np.abs(Bg - B) / np.maximum(np.abs(B), 1e-30))):.3e}")
            bitwise += 1
    assert bitwise == len(checkpoints)
    assert np.array_equal(a.B_final[0].cpu().numpy().view(np.uint32), B.view(np.uint32))
    g.close()


SHEET_VERSIONS = [v for v in VERSION_TABLE if v in orc.VERSIONS]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("V,M", [(64, 1024), (128, 1024)])
@pytest.mark.parametrize("version", SHEET_VERSIONS)
def test_every_version_320_epochs_against_oracle_from_scratch(version, V, M):
    """One (version, shape) trajectory of 320 epochs: the engine's run (one
    chunk, bond history) against orc.run from B = None. Reset versions get a
    reset at epoch 160 of column 5; for the conditional ones (C of the previous
    epoch == 0, simulation_utils.py:79-88) column 5 is zeroed at epoch 159 so
    the reset fires."""
    E = 320
    variant, reset = VERSION_TABLE[version]
    seed = 0x5EED0320 + V
    W = engine.synth_weights(seed, E, 1, V, M)
    S = torch.from_numpy(synth.stakes(seed, E, 1, V, period=40)).to(W.device)
    liquid = "liquid alpha on" in version
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=liquid))
    kw, rk = {}, {}
    if reset != engine.RESET_NONE:
        if reset == engine.RESET_IF_ZERO_CONSENSUS:
            W[159, ..., 5] = 0.0
        kw = {"reset_mode": reset, "reset_epoch": 160, "reset_index": 5, "n_miners": M, "n_epochs": E}
        rk = {"reset_epoch": 160, "reset_index": 5}
    params = [engine.make_params(variant, cfg, **kw)]
    a = engine.run(variant, params, W, S, want_hist=True)
    torch.cuda.synchronize()
    ref = orc.run(version, W[:, 0].cpu().numpy(), S[:, 0].cpu().numpy(), cfg, **rk)
    tag = f"{version} {V}x{M}"
    np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"], err_msg=tag)
    assert_close(a.Dn[:, 0].cpu().numpy(), ref["Dn"], what=f"{tag} Dn")
    assert_close(a.I[:, 0].cpu().numpy(), ref["I"], what=f"{tag} I")
    Bh = a.B_hist[:, 0].cpu().numpy()
    for t in range(E):
        assert_close(Bh[t], ref["B"][t], what=f"{tag} B[{t}]")
    if reset == engine.RESET_IF_ZERO_CONSENSUS:
        assert float(ref["C"][159][5]) == 0.0
