"""Wavelet coherence of two series (reference: src/wct.py).

``run_wct`` keeps the reference signature, including the misspelled keyword
``calculate_signficance`` (src/wct.py:96-140).  Coherence and phase arrows come from
the fused coherence kernels (``wtmi_wct_morlet``).  With significance off the
reference divides by ``signif = [0]`` and returns an all-inf ratio (quirk B.8);
that is reproduced.  Significance ON runs pycwt's Monte-Carlo ``wct_significance``
on the GPU (``transforms.wct_significance``: red noise K10, batched coherence,
counter K11; 300 passes, in-process cache like pycwt's ``cache=True``).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import List, Tuple, Type

import numpy as np
import numpy.typing as npt
import torch

from wtmi import ops, transforms
from wtmi.wavelets import DOG, MexicanHat, Morlet, Paul, as_morlet
from src.utils import wavelet_helpers

logger = logging.getLogger(__name__)

DT = 1 / 12
DJ = 1 / 8
S0 = 2 * DT
MOTHER = "morlet"
MOTHER_DICT = {  # coherence needs Morlet.smooth: the others raise (AttributeError, as pycwt.wct)
    "morlet": Morlet(6),
    "paul": Paul(),
    "DOG": DOG(),
    "mexicanhat": MexicanHat(),
}
LEVELS = [0.0625, 0.125, 0.25, 0.5, 1, 2, 4, 8, 16]
WCT_LEVELS = [0.0, 0.125, 0.25, 0.375, 0.5, 0.625, 0.75, 0.875, 1.0]

WCT_PLOT_PROPS = {
    "cmap": "jet", "sig_colors": "k", "sig_linewidths": 2, "coi_color": "k", "coi_alpha": 0.3,
    "coi_hatch": "--", "phase_diff_units": "width", "phase_diff_angles": "uv",
    "phase_diff_pivot": "mid", "phase_diff_linewidth": 0.5, "phase_diff_edgecolor": "k",
    "phase_diff_alpha": 0.7,
}


@dataclass
class DataForWCT:
    """Holds data for WCT"""

    t_values: npt.NDArray = field(init=False)
    y1_values: npt.NDArray
    y2_values: npt.NDArray
    mother_wavelet: Type
    delta_t: float
    delta_j: float
    initial_scale: float
    levels: List[float]
    actual_times: npt.NDArray = None

    def __post_init__(self):
        if self.actual_times is not None:
            self.t_values = self.actual_times
        else:
            self.t_values = np.linspace(1, self.y1_values.size + 1, self.y1_values.size)


@dataclass
class ResultsFromWCT:
    """Holds results from Wavelet Coherence Transform"""

    coherence: npt.NDArray
    period: npt.NDArray
    significance_levels: npt.NDArray
    coi: npt.NDArray
    phase_diff_u: npt.NDArray
    phase_diff_v: npt.NDArray


def run_wct(wavelet_coherence_transform: Type[DataForWCT], calculate_signficance: bool = True,
            significance_level: float = 0.95) -> Type[ResultsFromWCT]:
    """Coherence magnitude, period, significance ratio, cone of influence and phase."""
    d = wavelet_coherence_transform
    mother = as_morlet(d.mother_wavelet)
    y1, y2 = np.asarray(d.y1_values), np.asarray(d.y2_values)
    if y1.size != y2.size:
        raise AssertionError("Input signals must have the same size")
    d1 = transforms._to_dev(y1).reshape(1, -1)
    d2 = transforms._to_dev(y2).reshape(1, -1)
    x1 = ops.affine(d1, ops.series_affine(d1, ops.AFF_NORMALIZE), torch.float32)
    x2 = ops.affine(d2, ops.series_affine(d2, ops.AFF_NORMALIZE), torch.float32)
    res, sj, freqs = transforms.wct_batch(x1, x2, d.delta_t, d.delta_j, d.initial_scale, -1, mother,
                                          normalize=False, want_uv=True)
    n0 = y1.size
    coherence = transforms._np(res["coh"][0], np.float64)
    if calculate_signficance:
        # pycwt.wct(sig=True): AR(1) of the raw series, then the Monte-Carlo levels at
        # the transform's own resolution (J = -1 -> round(log2(n dt / s0) / dj))
        J = int(np.round(np.log2(n0 * d.delta_t / d.initial_scale) / d.delta_j))
        a1, _, _ = transforms.ar1(y1)
        a2, _, _ = transforms.ar1(y2)
        signif = transforms.wct_significance(a1, a2, d.delta_t, d.delta_j, d.initial_scale, J,
                                             significance_level=significance_level,
                                             wavelet=mother, cache=True)
    else:
        signif = np.asarray([0])
    with np.errstate(divide="ignore", invalid="ignore"):
        sig95 = np.abs(coherence) / (np.ones([1, n0]) * signif[:, None])
    coi = transforms.cone_of_influence(n0, d.delta_t, mother)
    u = transforms._np(res["u"][0], np.float64)
    v = transforms._np(res["v"][0], np.float64)
    return ResultsFromWCT(coherence, 1 / freqs, sig95, coi, u, v)


def calculate_phase_difference(wct_phase: npt.NDArray) -> Tuple[npt.NDArray, npt.NDArray]:
    angle = 0.5 * np.pi - wct_phase
    return np.cos(angle), np.sin(angle)


def plot_wct(wct_ax, wct_data: Type[DataForWCT], wct_results: Type[ResultsFromWCT],
             include_significance: bool = True, include_cone_of_influence: bool = True,
             include_phase_difference: bool = True, **kwargs) -> None:
    """Filled contours of |coherence| at WCT_LEVELS over (time, log2 period), the
    significance contour, the COI shading built like the CWT's ("cwt") and the phase
    arrows (src/wct.py:161-224)."""
    t, period = wct_data.t_values, wct_results.period
    wct_ax.contourf(t, np.log2(period), np.abs(wct_results.coherence), WCT_LEVELS,
                    extend="both", cmap=kwargs["cmap"],
                    extent=[min(t), max(t), min(wct_results.coi), max(period)])
    if include_significance:
        wavelet_helpers.plot_signficance_levels(wct_ax, wct_results.significance_levels, t,
                                                period, **kwargs)
    if include_cone_of_influence:
        wavelet_helpers.plot_cone_of_influence(wct_ax, wct_results.coi, t, wct_data.levels, period,
                                               wct_data.delta_t, tranform_type="cwt", **kwargs)
    if include_phase_difference:
        plot_phase_difference(wct_ax, t, period, wct_results.phase_diff_u,
                              wct_results.phase_diff_v, **kwargs)


def plot_phase_difference(wct_ax, t_values: npt.NDArray, period: npt.NDArray,
                          phase_diff_u: npt.NDArray, phase_diff_v: npt.NDArray, **kwargs) -> None:
    """Phase arrows thinned to about 48 columns x 12 rows (src/wct.py:227-265)."""
    rows, cols = phase_diff_u.shape
    ys, xs = max(1, rows // 12), max(1, cols // 48)
    wct_ax.quiver(t_values[::xs], np.log2(period[::ys]),
                  phase_diff_u[::ys, ::xs], phase_diff_v[::ys, ::xs],
                  units=kwargs["phase_diff_units"], angles=kwargs["phase_diff_angles"],
                  pivot=kwargs["phase_diff_pivot"], linewidth=kwargs["phase_diff_linewidth"],
                  edgecolor=kwargs["phase_diff_edgecolor"], alpha=kwargs["phase_diff_alpha"])
