"""Dividend arithmetic and matplotlib charts for the chart table.

``_calculate_total_dividends`` is used by the dividend sheet (reference
charts_utils.py:15-45); the plotting helpers are the rendering side of
v1.api.generate_chart_table and stay on the CPU.
"""

from __future__ import annotations


def _calculate_total_dividends(
    validators: list[str],
    dividends_per_validator: dict[str, list[float]],
    base_validator: str,
    num_epochs: int,
) -> tuple[dict[str, float], dict[str, float]]:
    """Total dividend per validator over the first `num_epochs` epochs, and the
    percentage difference of each to `base_validator` (reference :15-45)."""
    totals = {v: sum(dividends_per_validator.get(v, [])[:num_epochs]) for v in validators}
    base = totals.get(base_validator)
    if base is None or base == 0.0:
        print(f"Warning: Base validator '{base_validator}' has zero or missing total dividends.")
        base = 1e-6
    diffs = {
        v: 0.0 if v == base_validator else (total - base) / base * 100.0
        for v, total in totals.items()
    }
    return totals, diffs


# ---------------------------------------------------------------------------
# matplotlib rendering (CPU; reference charts_utils.py:48-398)
# ---------------------------------------------------------------------------
import base64  # noqa: E402
import io  # noqa: E402

import numpy as np  # noqa: E402

_STYLES = (("-", "+", 12, 2), ("--", "x", 12, 1), (":", "o", 4, 1))


def _plt():
    import matplotlib

    matplotlib.use("Agg", force=False)
    import matplotlib.pyplot as plt

    return plt


def _get_validator_styles(validators: list[str]) -> dict[str, tuple[str, str, int, int]]:
    """(linestyle, marker, markersize, markeredgewidth) per validator, cycling."""
    return {v: _STYLES[i % len(_STYLES)] for i, v in enumerate(validators)}


def _set_default_xticks(ax, num_epochs: int) -> None:
    locs = [0, 1, 2] + list(range(5, num_epochs, 5))
    ax.set_xticks(locs)
    ax.set_xticklabels([str(i) for i in locs], fontsize=8)


def _plot_to_base64() -> str:
    """Render the current figure as an inline PNG <img> tag."""
    plt = _plt()
    buf = io.BytesIO()
    plt.savefig(buf, format="png", transparent=True, bbox_inches="tight", dpi=100)
    plt.close()
    data = base64.b64encode(buf.getvalue()).decode("ascii")
    return f'<img src="data:image/png;base64,{data}" style="max-width:1200px; height:auto;" draggable="false">'


def _finish(to_base64: bool):
    if to_base64:
        return _plot_to_base64()
    _plt().show()
    return None


def _plot_dividends(num_epochs, validators, dividends_per_validator, case, base_validator,
                    to_base64: bool = False):
    """Dividend per 1000 tao per epoch for each validator, with totals and the
    percentage difference to the base validator in the legend."""
    plt = _plt()
    plt.close("all")
    _, ax = plt.subplots(figsize=(14, 6))
    styles = _get_validator_styles(validators)
    totals, diffs = _calculate_total_dividends(validators, dividends_per_validator, base_validator, num_epochs)
    n = None
    for idx, (v, divs) in enumerate(dividends_per_validator.items()):
        y = np.asarray([float(d) for d in divs], dtype=float)
        if n is None:
            n = len(y)
        x = np.arange(len(y)) + idx * 0.05
        ls, mk, ms, mew = styles[v]
        pct = diffs[v]
        tag = "(Base)" if pct == 0 else (f"(+{pct:.1f}%)" if pct > 0 else f"({pct:.1f}%)")
        ax.plot(x, y, marker=mk, markeredgewidth=mew, markersize=ms, linestyle=ls, alpha=0.7,
                label=f"{v}: Total = {totals[v]:.6f} {tag}")
    if n is not None:
        _set_default_xticks(ax, n)
    ax.set_xlabel("Time (Epochs)")
    ax.set_ylim(bottom=0)
    ax.set_ylabel("Dividend per 1,000 Tao per Epoch")
    ax.set_title(case)
    ax.grid(True)
    ax.legend()
    if case.startswith("Case 4"):
        ax.set_ylim(0, 0.042)
    plt.subplots_adjust(hspace=0.3)
    return _finish(to_base64)


def _prepare_bond_data(bonds_per_epoch, validators, servers, normalize: bool):
    """bonds[server][validator] -> per-epoch list; optionally each epoch's
    column normalised to sum 1 (when the column sum exceeds 1e-12)."""
    stack = np.stack([np.asarray(b.detach().cpu() if hasattr(b, "detach") else b, dtype=float)
                      for b in bonds_per_epoch]) if bonds_per_epoch else np.zeros((0, len(validators), len(servers)))
    data = [[list(stack[:, iv, js]) for iv in range(len(validators))] for js in range(len(servers))]
    if normalize:
        for js in range(len(servers)):
            for e in range(stack.shape[0]):
                tot = sum(data[js][iv][e] for iv in range(len(validators)))
                if tot > 1e-12:
                    for iv in range(len(validators)):
                        data[js][iv][e] /= tot
    return data


def _plot_bonds(num_epochs, validators, servers, bonds_per_epoch, case_name, to_base64: bool = False,
                normalize: bool = False):
    """Bond value (or ratio) per server for each validator."""
    plt = _plt()
    fig, axes = plt.subplots(1, len(servers), figsize=(14, 5), sharex=True, sharey=True)
    axes = [axes] if len(servers) == 1 else list(axes)
    data = _prepare_bond_data(bonds_per_epoch, validators, servers, normalize)
    styles = _get_validator_styles(validators)
    handles, labels = [], []
    x = list(range(num_epochs))
    for js, server in enumerate(servers):
        ax = axes[js]
        for iv, v in enumerate(validators):
            ls, mk, ms, mew = styles[v]
            (line,) = ax.plot(x, data[js][iv], alpha=0.7, marker=mk, markersize=ms, markeredgewidth=mew,
                              linestyle=ls, linewidth=2)
            if js == 0:
                handles.append(line)
                labels.append(v)
        _set_default_xticks(ax, num_epochs)
        ax.set_xlabel("Epoch")
        if js == 0:
            ax.set_ylabel("Bond Ratio" if normalize else "Bond Value")
        ax.set_title(server)
        ax.grid(True)
        if normalize:
            ax.set_ylim(0, 1.05)
    fig.suptitle(f"Validators bonds per Server{' normalized' if normalize else ''}\n{case_name}", fontsize=14)
    fig.legend(handles, labels, loc="lower center", ncol=len(validators), bbox_to_anchor=(0.5, 0.02))
    plt.tight_layout(rect=(0, 0.05, 0.98, 0.95))
    return _finish(to_base64)


def _plot_validator_server_weights(validators, weights_epochs, servers, num_epochs, case_name,
                                   to_base64: bool = False):
    """Each validator's weight on server 2 over time, server names on the axis
    ends and percentage ticks for intermediate levels."""
    plt = _plt()
    styles = _get_validator_styles(validators)
    series = [[float(weights_epochs[e][iv][1]) for e in range(num_epochs)] for iv in range(len(validators))]
    ticks = {0.0: servers[0], 1.0: servers[1]}
    for y in sorted({y for s in series for y in s}):
        if y in (0.0, 1.0) or min(abs(y), abs(y - 1.0)) < 0.02:
            continue
        if all(abs(y - t) >= 0.05 for t in ticks):
            pct = y * 100
            ticks[y] = f"{pct:.0f}%" if float(pct).is_integer() else f"{pct:.1f}%"
    pos = sorted(ticks)
    fig, ax = plt.subplots(figsize=(14, 1 if len(pos) <= 2 else 3))
    ax.set_ylim(-0.05, 1.05)
    for iv, v in enumerate(validators):
        ls, mk, ms, mew = styles[v]
        ax.plot(range(num_epochs), series[iv], label=v, marker=mk, linestyle=ls, markersize=ms,
                markeredgewidth=mew, linewidth=2)
    ax.set_yticks(pos)
    ax.set_yticklabels([ticks[p] for p in pos])
    _set_default_xticks(ax, num_epochs)
    ax.set_xlabel("Epoch")
    ax.set_title(f"Validators Weights to Servers \n{case_name}")
    ax.legend()
    ax.grid(True)
    return _finish(to_base64)


def _plot_incentives(servers, server_incentives_per_epoch, num_epochs, case_name, to_base64: bool = False):
    """Server incentive per epoch."""
    plt = _plt()
    _, ax = plt.subplots(figsize=(14, 3))
    x = np.arange(num_epochs)
    for js, server in enumerate(servers):
        ax.plot(x, [float(inc[js]) for inc in server_incentives_per_epoch], label=server)
    _set_default_xticks(ax, num_epochs)
    ax.set_xlabel("Epoch")
    ax.set_ylabel("Server Incentive")
    ax.set_title(f"Server Incentives\n{case_name}")
    ax.set_ylim(-0.05, 1.05)
    ax.legend()
    ax.grid(True)
    return _finish(to_base64)
