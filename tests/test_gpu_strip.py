"""The column-normalised strip scan k_bonds_cn (YumaRust above 64
validators; Yuma / Yuma2 when the full outputs turn the rank-formed column
sums off) at every rows-per-lane form: R = 1 (<= 128 validators), 2 (<= 256),
4 (<= 512), 8 (<= 1024), across several LDS flushes of the parked dividend
partials (32 / 32 / 16 / 8 epochs), against the oracle's epoch loop from
scratch (yumas.py:113-153, :227-262; simulation_utils.py:44-110): C exact,
Dn / I / B within 1e-5 at every epoch. Odd V leaves padding rows in the last
row set; one case feeds a row outside the division screen (k_rowsum's
reciprocal is NaN: the wave's IEEE path)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import assert_close
from oracle import yuma_oracle as orc

pytestmark = pytest.mark.gpu

from yuma_simulation._internal import engine, synth  # noqa: E402
from yuma_simulation._internal.yumas import YumaConfig, YumaParams  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "gpu tests need a ROCm GPU"
    engine.load_library()
    yield
    torch.cuda.empty_cache()


VERSIONS = {engine.VARIANT_RUST: "Yuma 0 (subtensor)", engine.VARIANT_YUMA1: "Yuma 1 (paper)",
            engine.VARIANT_YUMA2: "Yuma 2 (Adrian-Fish)"}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("variant,V,E,liquid,want,tiny", [
    (engine.VARIANT_RUST, 100, 70, False, (), False),
    (engine.VARIANT_RUST, 256, 70, True, (), False),
    (engine.VARIANT_RUST, 300, 40, False, (), False),
    (engine.VARIANT_RUST, 700, 20, True, (), False),
    (engine.VARIANT_RUST, 1000, 20, False, (), False),
    (engine.VARIANT_RUST, 200, 36, False, (), True),
    # Yuma / Yuma2 with W_n requested: the rank pass forms no column sums,
    # the bond scan is k_bonds_cn
    (engine.VARIANT_YUMA1, 300, 40, False, ("Wn",), False),
    (engine.VARIANT_YUMA2, 130, 40, True, ("Wn",), False),
])
def test_strip_scan_against_oracle(variant, V, E, liquid, want, tiny):
    M = 512
    seed = 0x57A1 + V
    W = synth.weights(seed, E, 1, V, M)
    S = synth.stakes(seed, E, 1, V, period=9)
    if tiny:
        # one row with a weight below 2^-60 after normalisation: k_rowsum's
        # screen fails for it (rq4.y NaN) and its waves divide by IEEE
        W[3, 0, 7, :] = 0.0
        W[3, 0, 7, 5] = np.float32(1e-30)
        W[3, 0, 7, 9] = np.float32(1.0)
    cfg = YumaConfig(yuma_params=YumaParams(liquid_alpha=liquid))
    params = [engine.make_params(variant, cfg)]
    a = engine.run(variant, params, torch.from_numpy(W), torch.from_numpy(S), want_hist=True, want=want)
    torch.cuda.synchronize()
    version = VERSIONS[variant] + (" - liquid alpha on" if liquid and variant == engine.VARIANT_YUMA1 else "")
    ref = orc.run(version, W[:, 0], S[:, 0], cfg)
    tag = f"{version} V={V}"
    np.testing.assert_array_equal(a.C[:, 0].cpu().numpy(), ref["C"], err_msg=tag)
    assert_close(a.Dn[:, 0].cpu().numpy(), ref["Dn"], what=f"{tag} Dn")
    assert_close(a.I[:, 0].cpu().numpy(), ref["I"], what=f"{tag} I")
    Bh = a.B_hist[:, 0].cpu().numpy()
    for t in range(E):
        assert_close(Bh[t], ref["B"][t], what=f"{tag} B[{t}]")
    assert_close(a.B_final[0].cpu().numpy(), ref["B"][-1], what=f"{tag} B_final")
