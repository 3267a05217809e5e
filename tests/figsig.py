"""Figure signatures: what a plot function drew, as comparable plain data.

Shared by ``scripts/make_plot_golden.py`` (runs the reference's own plot functions in the
build container and stores their signatures in ``tests/golden/plot_signatures.json``) and
``tests/test_plots.py`` (runs the repo's plot functions on the same inputs).  Inputs are
synthetic and seeded (``plot_inputs``), so both sides see identical arrays.
"""

from __future__ import annotations

import types

import numpy as np


def _sum(a):
    a = np.asarray(a, dtype=np.float64)
    return [list(a.shape), float(np.nansum(a)), float(np.nansum(np.abs(a)))]


def _collection(c):
    d = {"type": type(c).__name__}
    if hasattr(c, "levels"):  # ContourSet (filled or lines)
        d["levels"] = [float(v) for v in c.levels]
        d["filled"] = bool(getattr(c, "filled", False))
        d["extend"] = getattr(c, "extend", None)
        paths = c.get_paths()
        d["n_paths"] = len(paths)
        verts = [p.vertices for p in paths if len(p.vertices)]
        d["vertices"] = _sum(np.concatenate(verts)) if verts else None
        d["linewidths"] = [float(v) for v in np.atleast_1d(c.get_linewidth())][:4]
    if type(c).__name__ == "Quiver":
        d["N"] = int(c.N)
        d["U"], d["V"] = _sum(c.U), _sum(c.V)
        d["XY"] = _sum(c.XY)
        d["units"], d["angles"], d["pivot"] = c.units, c.angles, c.pivot
        d["alpha"] = c.get_alpha()
    return d


def _patch(p):
    d = {"type": type(p).__name__, "alpha": p.get_alpha(), "hatch": p.get_hatch()}
    if hasattr(p, "get_xy"):
        d["xy"] = _sum(p.get_xy())
    d["facecolor"] = [round(float(v), 6) for v in p.get_facecolor()]
    return d


def _line(ln):
    return {"label": ln.get_label() if not ln.get_label().startswith("_") else None,
            "x": _sum(ln.get_xdata()), "y": _sum(ln.get_ydata())}


def axes_signature(ax):
    leg = ax.get_legend()
    return {
        "title": ax.get_title(),
        "xlim": [float(v) for v in ax.get_xlim()],
        "ylim": [float(v) for v in ax.get_ylim()],
        "yticks": [float(v) for v in ax.get_yticks()],
        "yticklabels": [t.get_text() for t in ax.get_yticklabels()],
        "collections": [_collection(c) for c in ax.collections],
        "patches": [_patch(p) for p in ax.patches],
        "lines": [_line(ln) for ln in ax.lines],
        "legend": None if leg is None else {
            "texts": [t.get_text() for t in leg.get_texts()], "frameon": leg.get_frame_on()},
    }


def figure_signature(fig):
    return [axes_signature(ax) for ax in fig.axes]


def compare(got, want, path="fig", rtol=1e-9):
    """Raise AssertionError naming the first difference (floats to rtol)."""
    if isinstance(want, dict):
        assert isinstance(got, dict) and sorted(got) == sorted(want), (path, got, want)
        for k in want:
            compare(got[k], want[k], f"{path}.{k}", rtol)
    elif isinstance(want, list):
        assert isinstance(got, list) and len(got) == len(want), (path, got, want)
        for i, (g, w) in enumerate(zip(got, want)):
            compare(g, w, f"{path}[{i}]", rtol)
    elif isinstance(want, float):
        assert isinstance(got, (float, int)), (path, got, want)
        assert abs(got - want) <= rtol * max(1.0, abs(want)), (path, got, want)
    else:
        assert got == want, (path, got, want)


PLOT_PROPS = {  # the app's own plot properties (constants/results_configs.py:41-70)
    "cmap": "jet", "sig_colors": "k", "sig_linewidths": 2, "coi_color": "k", "coi_alpha": 0.3,
    "coi_hatch": "--", "phase_diff_units": "width", "phase_diff_angles": "uv",
    "phase_diff_pivot": "mid", "phase_diff_linewidth": 0.5, "phase_diff_edgecolor": "k",
    "phase_diff_alpha": 0.7,
}
LEVELS = [0.0625, 0.125, 0.25, 0.5, 1, 2, 4, 8, 16]


def plot_inputs(seed=0):
    """Synthetic, seeded stand-ins for the transform results each plot function reads
    (n = 240 monthly samples; 85 CWT scales; 62 XWT / 93 phase rows (dj 1/8 vs 1/12);
    a 5-level DWT coefficient list and smoothing dict)."""
    rng = np.random.default_rng(seed)
    n, dt = 240, 1 / 12
    t_years = np.arange(1, n + 1) * dt + 1990
    S = 85
    period = 2 * dt * 1.033 * 2 ** (np.arange(S) / 12)
    coi = 1.033 / np.sqrt(2) * dt * (n / 2 - np.abs(np.arange(n) - (n - 1) / 2))
    coi[0] = coi[-1] = 1e-5
    cwt_data = types.SimpleNamespace(time_range=t_years, levels=LEVELS, delta_t=dt)
    cwt_res = types.SimpleNamespace(power=rng.gamma(1.0, 1.0, (S, n)) * 2.0, period=period,
                                    significance_levels=rng.gamma(1.0, 1.0, (S, n)), coi=coi)
    Sx, Sp = 62, 93
    t_lin = np.linspace(1, n + 1, n)
    period_x = 2 * dt * 1.033 * 2 ** (np.arange(Sx) / 8)
    coi_poly = np.concatenate([np.log2(coi), [1e-9], np.log2(period_x[-1:]),
                               np.log2(period_x[-1:]), [1e-9]]).clip(min=np.log2(LEVELS[2]))
    ph = rng.uniform(-np.pi, np.pi, (Sp, n))
    xwt_data = types.SimpleNamespace(t_values=t_lin, levels=LEVELS, delta_t=dt)
    xwt_res = types.SimpleNamespace(power=rng.gamma(1.0, 1.0, (Sx, n)), period=period_x,
                                    significance_levels=rng.gamma(1.0, 1.0, (Sx, n)),
                                    coi=coi_poly, phase_diff_u=np.sin(ph), phase_diff_v=np.cos(ph))
    phw = rng.uniform(-np.pi, np.pi, (Sx, n))
    wct_res = types.SimpleNamespace(coherence=rng.uniform(0, 1, (Sx, n)), period=period_x,
                                    significance_levels=rng.uniform(0, 2, (Sx, n)), coi=coi,
                                    phase_diff_u=np.sin(phw), phase_diff_v=np.cos(phw))
    y = rng.standard_normal(n).cumsum()
    lens = [14, 14, 21, 36, 65, 123]  # pywt db4 symmetric, n = 240, level 5
    coeffs = [rng.standard_normal(k) for k in lens]
    smooth = {lvl: {"signal": y + 0.1 * lvl * rng.standard_normal(n)} for lvl in range(5, 0, -1)}
    return {"n": n, "t_years": t_years, "cwt": (cwt_data, cwt_res), "xwt": (xwt_data, xwt_res),
            "wct": (xwt_data, wct_res), "y": y, "coeffs": coeffs, "smooth": smooth}
