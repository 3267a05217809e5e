"""Cross-wavelet transform of two series (reference: src/xwt.py).

``run_xwt`` keeps the reference signature (src/xwt.py:83-139).  Power |W1 W2*|^2 and
the significance ratio come from one pair-mode HIP kernel launch; the phase arrows
from a second launch at the scales pycwt.wct would use -- the reference passes
``delta_j=`` to ``wct`` which swallows it, so the phase runs at dj = 1/12
(quirk B.5).  ``run_xwt`` fails where the reference fails: ``normalize=False`` raises
NameError (B.7) and non-Morlet mothers (``MOTHER_DICT["paul"]``, ``["DOG"]``,
``["mexicanhat"]``) raise AttributeError, as pycwt.wct does for a mother without
``smooth``.  The engine extension ``run_xwt_batch`` offers both as explicit options:
``normalize=False`` returns the raw complex cross spectrum, and
``phase_without_smooth=True`` gives the non-Morlet mothers pycwt.xwt's power and
significance with phase arrows from the angle of W1 W2* (what pycwt.wct returns as aWCT,
which needs no smoothing).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import List, Tuple, Type

import numpy as np
import numpy.typing as npt
import torch

from wtmi import ops, transforms
from wtmi.wavelets import DOG, MexicanHat, Morlet, Paul, as_morlet, as_mother, kernel_mother
from src.utils import wavelet_helpers
from src.utils.wavelet_helpers import coi_polygon

logger = logging.getLogger(__name__)

DT = 1 / 12
DJ = 1 / 8
S0 = 2 * DT
MOTHER = "morlet"
MOTHER_DICT = {  # every key is transformable (the CWT kernels evaluate each mother's filter)
    "morlet": Morlet(6),
    "paul": Paul(),
    "DOG": DOG(),
    "mexicanhat": MexicanHat(),
}
LEVELS = [0.0625, 0.125, 0.25, 0.5, 1, 2, 4, 8, 16]

XWT_PLOT_PROPS = {
    "cmap": "jet", "sig_colors": "k", "sig_linewidths": 2, "coi_color": "k", "coi_alpha": 0.3,
    "coi_hatch": "--", "phase_diff_units": "width", "phase_diff_angles": "uv",
    "phase_diff_pivot": "mid", "phase_diff_linewidth": 0.5, "phase_diff_edgecolor": "k",
    "phase_diff_alpha": 0.7,
}


@dataclass
class DataForXWT:
    """Holds data for XWT"""

    t_values: npt.NDArray = field(init=False)
    y1_values: npt.NDArray
    y2_values: npt.NDArray
    mother_wavelet: Type
    delta_t: float
    delta_j: float
    initial_scale: float
    levels: List[float]

    def __post_init__(self):
        self.t_values = np.linspace(1, self.y1_values.size + 1, self.y1_values.size)


@dataclass
class ResultsFromXWT:
    """Holds results from Cross-Wavelet Transform"""

    power: npt.NDArray
    period: npt.NDArray
    significance_levels: npt.NDArray
    coi: npt.NDArray
    phase_diff_u: npt.NDArray
    phase_diff_v: npt.NDArray


def run_xwt(cross_wavelet_transform: Type[DataForXWT], normalize: bool = True
            ) -> Type[ResultsFromXWT]:
    """Cross-wavelet power, period, significance ratio, COI polygon and phase arrows.

    As the reference does: ``normalize=False`` raises NameError (its else branch reads
    ``signal_size``, bound only under ``normalize``; quirk B.7), and a Paul / DOG /
    MexicanHat mother raises AttributeError (pycwt.wct has no ``smooth`` for it).  The
    engine's alternatives are explicit: ``run_xwt_batch(..., normalize=False)`` (raw cross
    spectrum) and ``run_xwt_batch(..., phase_without_smooth=True)``."""
    if not normalize:
        raise NameError("name 'signal_size' is not defined")
    return run_xwt_batch([cross_wavelet_transform], normalize=normalize)[0]


def run_xwt_batch(xwt_data_list: List[DataForXWT], normalize: bool = True,
                  phase_without_smooth: bool = False) -> List[ResultsFromXWT]:
    """``run_xwt`` over many pairs (engine extension; the reference loops in
    src/utils/transform_helpers.py:126-135).  Pairs of one length and transform
    parameters share one normalisation, one pair-mode XWT launch (per-pair AR(1)
    significance as a [B, S] multiplier) and one phase launch.

    The reference takes the phase arrows from pycwt.wct (src/xwt.py:122-134), which needs
    ``wavelet.smooth`` -- Morlet's only -- so for Paul / DOG / MexicanHat it raises
    AttributeError, and so does this function by default (before any launch; the reference
    would raise after its xwt, which has no side effect).  ``phase_without_smooth=True`` is
    the engine's explicit alternative: the arrows from angle(W1 W2*) at dj = 1/12, which is
    what pycwt.wct returns as aWCT and needs no smoothing."""
    if not phase_without_smooth:
        for d in xwt_data_list:
            if kernel_mother(d.mother_wavelet)[0] != 0:
                as_morlet(d.mother_wavelet)  # raises NoSmoothError (an AttributeError), as pycwt.wct
    out: List[ResultsFromXWT] = [None] * len(xwt_data_list)
    groups: dict = {}
    for i, d in enumerate(xwt_data_list):
        n1, n2 = np.asarray(d.y1_values).size, np.asarray(d.y2_values).size
        if n1 != n2:
            raise ValueError("y1_values and y2_values must have the same length")
        key = (n1, kernel_mother(d.mother_wavelet), float(d.delta_t), float(d.delta_j),
               float(d.initial_scale), tuple(d.levels))
        groups.setdefault(key, []).append(i)
    for (n0, _, dt, dj, s0, levels), idx in groups.items():
        mother = as_mother(xwt_data_list[idx[0]].mother_wavelet)
        d1 = transforms._to_dev(np.stack([np.asarray(xwt_data_list[i].y1_values, dtype=np.float64)
                                          for i in idx]))
        d2 = transforms._to_dev(np.stack([np.asarray(xwt_data_list[i].y2_values, dtype=np.float64)
                                          for i in idx]))
        m1, m2 = ops.series_moments(d1), ops.series_moments(d2)
        # pycwt.xwt(normalize=True): (y - mean) / std, in fp64 on the GPU
        x1 = ops.affine(d1, transforms.normalize_coefs(m1), torch.float32)
        x2 = ops.affine(d2, transforms.normalize_coefs(m2), torch.float32)
        sj, freqs = transforms.scales_for(n0, dt, dj, s0, -1, mother)
        mh1, mh2 = transforms._np(m1), transforms._np(m2)
        dof = mother.dofmin
        chi = transforms._chi2_ppf(0.95, dof) / dof  # DOG: dofmin 1
        signif = []
        for k in range(len(idx)):
            g1, _, _ = transforms._ar1_from_moments(mh1[k, 4], mh1[k, 5], int(mh1[k, 6]))
            g2, _, _ = transforms._ar1_from_moments(mh2[k, 4], mh2[k, 5], int(mh2[k, 6]))
            Pk1 = transforms.ar1_spectrum(freqs * dt, g1)
            Pk2 = transforms.ar1_spectrum(freqs * dt, g2)
            # the reference calls pycwt.xwt with its default normalize=True whatever run_xwt's
            # own flag (src/xwt.py:93-101), and pycwt then resets std1 = std2 = 1
            signif.append((Pk1 * Pk2) ** 0.5 * chi)
        signif = np.stack(signif)
        period = 1 / freqs
        coi = transforms.cone_of_influence(n0, dt, mother)
        if normalize:
            r = ops.xwt_morlet(x1, x2, sj, dt, sig_scale=1.0 / signif, want_power=True,
                               want_sig=True, mother=mother)
            power = transforms._np(r["power"], np.float64)
            sig95 = transforms._np(r["sig"], np.float64)
            coi_plot = coi_polygon(coi, period, np.log2(levels[2]))
        else:
            r = ops.xwt_morlet(x1, x2, sj, dt, want_w12=True, mother=mother)
            power = transforms._np(r["w12"], np.complex128)
            sig95 = power / (np.ones([1, n0]) * signif[:, :, None])
            coi_plot = coi
        # phase: pycwt.wct(..., delta_j=...) runs at its default dj = 1/12 (quirk B.5)
        sj_p, _ = transforms.scales_for(n0, dt, 1 / 12, s0, -1, mother)
        rp = ops.xwt_morlet(x1, x2, sj_p, dt, want_uv=True, mother=mother)
        u = transforms._np(rp["u"], np.float64)
        v = transforms._np(rp["v"], np.float64)
        for k, i in enumerate(idx):
            out[i] = ResultsFromXWT(power[k], period.copy(), sig95[k], coi_plot.copy(), u[k], v[k])
    return out


def calculate_phase_difference(xwt_phase: npt.NDArray) -> Tuple[npt.NDArray, npt.NDArray]:
    """Arrow components (Torrence & Webster 1999): u = cos(pi/2 - phase), v = sin(...)."""
    angle = 0.5 * np.pi - xwt_phase
    return np.cos(angle), np.sin(angle)


def plot_xwt(xwt_ax, xwt_data: Type[DataForXWT], xwt_results: Type[ResultsFromXWT],
             include_significance: bool = True, include_cone_of_influence: bool = True,
             include_phase_difference: bool = True, **kwargs) -> None:
    """Filled contours of log2 cross power at log2(levels) over (time, log2 period),
    then the significance contour, the COI polygon (already in log2 space, "xwt") and
    the phase arrows (src/xwt.py:157-223)."""
    t, period = xwt_data.t_values, xwt_results.period
    xwt_ax.contourf(t, np.log2(period), np.log2(xwt_results.power), np.log2(xwt_data.levels),
                    extend="both", cmap=kwargs["cmap"],
                    extent=[min(t), max(t), min(xwt_results.coi), max(period)])
    if include_significance:
        wavelet_helpers.plot_signficance_levels(xwt_ax, xwt_results.significance_levels, t,
                                                period, **kwargs)
    if include_cone_of_influence:
        wavelet_helpers.plot_cone_of_influence(xwt_ax, xwt_results.coi, t, xwt_data.levels, period,
                                               xwt_data.delta_t, tranform_type="xwt", **kwargs)
    if include_phase_difference:
        plot_phase_difference(xwt_ax, t, period, xwt_results.phase_diff_u,
                              xwt_results.phase_diff_v, **kwargs)


def plot_phase_difference(xwt_ax, t_values: npt.NDArray, period: npt.NDArray,
                          phase_diff_u: npt.NDArray, phase_diff_v: npt.NDArray, **kwargs) -> None:
    """Phase arrows on a fixed decimation: every 12th sample, every 8th period and
    every 12th row of u/v (src/xwt.py:226-253).  The u/v rows are at dj = 1/12 and the
    periods at dj = 1/8 (quirk B.5), so the two decimations select the same number of
    rows.  kwargs: ``phase_diff_{units,angles,pivot,linewidth,edgecolor,alpha}``."""
    xwt_ax.quiver(t_values[::12], np.log2(period[::8]),
                  phase_diff_u[::12, ::12], phase_diff_v[::12, ::12],
                  units=kwargs["phase_diff_units"], angles=kwargs["phase_diff_angles"],
                  pivot=kwargs["phase_diff_pivot"], linewidth=kwargs["phase_diff_linewidth"],
                  edgecolor=kwargs["phase_diff_edgecolor"], alpha=kwargs["phase_diff_alpha"])
