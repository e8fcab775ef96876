"""The public chart-table API (v1.api.generate_chart_table), mirroring the
reference's only computational test (tests/unit/api/api_test.py:8-26: all
14 cases, Yuma 1, bond_penalty 0.99, every <img> a base64 PNG) on the HIP
engine, plus the memoisation and duplicate-version behaviour of api.py."""

from __future__ import annotations

from html.parser import HTMLParser

import pytest
import torch

from yuma_simulation._internal import simulation_utils
from yuma_simulation._internal.cases import cases
from yuma_simulation._internal.yumas import SimulationHyperparameters, YumaParams, YumaSimulationNames
from yuma_simulation.v1 import api

pytestmark = pytest.mark.gpu


class _Imgs(HTMLParser):
    def __init__(self):
        super().__init__()
        self.srcs: list[str] = []
        self.headers: list[str] = []
        self._th = False

    def handle_starttag(self, tag, attrs):
        if tag == "img":
            self.srcs.append(dict(attrs).get("src", ""))
        self._th = tag == "th"

    def handle_data(self, data):
        if self._th:
            self.headers.append(data)
            self._th = False


def _parse(html_obj) -> _Imgs:
    p = _Imgs()
    p.feed(html_obj.data)
    return p


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs the HIP engine")


def test_generate_chart_table_with_charts(monkeypatch):
    """reference tests/unit/api/api_test.py:8-26, plus: the simulations run
    once (one batched run_simulations call), not once per chart type."""
    calls = []
    real = api.run_simulations

    def spy(runs, **kw):
        calls.append(len(runs))
        return real(runs, **kw)

    monkeypatch.setattr(api, "run_simulations", spy)
    names = YumaSimulationNames()
    table = api.generate_chart_table(cases, [(names.YUMA, YumaParams())],
                                     SimulationHyperparameters(bond_penalty=0.99))
    imgs = _parse(table)
    assert len(imgs.srcs) > 0, "Should contain at least one chart image"
    for src in imgs.srcs:
        assert src.startswith("data:image/png;base64,"), "Image should be base64-encoded"
    # 4 charts per case, 5 for the cases at index 9 and 10 (reference v1/api.py:42-45)
    assert len(imgs.srcs) == 4 * len(cases) + 2
    assert calls == [len(cases)]


def test_chart_table_duplicate_version_keeps_one_column():
    """A version listed twice keeps one column (the reference keys each row by
    version, reference v1/api.py:34-36, 50-119): the table builds, with one image per chart row."""
    names = YumaSimulationNames()
    two = [(names.YUMA, YumaParams()), (names.YUMA3, YumaParams()), (names.YUMA, YumaParams(bond_alpha=0.2))]
    table = api.generate_chart_table(cases[:2], two, SimulationHyperparameters(bond_penalty=0.99),
                                     draggable_table=True)
    imgs = _parse(table)
    assert imgs.headers == [names.YUMA, names.YUMA3]
    assert len(imgs.srcs) == 2 * 4 * 2
