"""Continuous wavelet transform of one series (reference: src/cwt.py).

Same constants, dataclasses and ``run_cwt`` signature as the reference
(src/cwt.py:37-135); the transform, |W|^2 and the significance ratio are produced
by one fused HIP kernel (``wtmi_cwt_morlet``), standardisation and the AR(1)
covariances by the moments/affine kernels.  Reference quirks kept:
``normalize`` is a no-op (B.1), AR(1) uses ``y_values`` not the standardised series
(B.2), significance uses variance 1.0 and the module constants DT/DJ/S0/J (B.3).
"""

from __future__ import annotations

import logging
from dataclasses import dataclass, field
from typing import List, Type

import numpy as np
import numpy.typing as npt
import torch

from wtmi import ops, transforms
from wtmi.wavelets import Morlet, as_mother, kernel_mother
from src.utils.wavelet_helpers import plot_cone_of_influence, plot_signficance_levels

logger = logging.getLogger(__name__)

UNITS = "%"
NORMALIZE = True
DT = 1 / 12  # In years
S0 = 2 * DT  # Starting scale
DJ = 1 / 12  # Twelve sub-octaves per octaves
J = 7 / DJ  # Seven powers of two with DJ sub-octaves
MOTHER = Morlet(f0=6)
LEVELS = [0.0625, 0.125, 0.25, 0.5, 1, 2, 4, 8, 16]


@dataclass
class DataForCWT:
    """Holds data for continuous wavelet transform"""

    t_values: npt.NDArray
    y_values: npt.NDArray
    mother_wavelet: Type
    delta_t: float
    delta_j: float
    initial_scale: float
    levels: List[float]
    time_range: npt.NDArray = field(init=False)

    def __post_init__(self):
        # reference quirk B.4: the method is shadowed by its own result
        self.time_range = self.time_range(self)

    def time_range(self) -> npt.NDArray:
        t0 = min(self.t_values)
        t0 = t0.astype("datetime64[Y]").astype(int) + 1970
        num_observations = self.t_values.size
        self.time_range = np.arange(1, num_observations + 1) * self.delta_t + t0
        return np.arange(1, num_observations + 1) * self.delta_t + t0


@dataclass
class ResultsFromCWT:
    """Holds results from continuous wavelet transform"""

    power: npt.NDArray
    period: npt.NDArray
    significance_levels: npt.NDArray
    coi: npt.NDArray


def run_cwt(cwt_data: Type[DataForCWT], normalize: bool = True, standardize: bool = False,
            calculate_significance: bool = True, significance_level: float = 0.95,
            **kwargs) -> Type[ResultsFromCWT]:
    """Conducts Continuous Wavelet Transform.
    Returns power spectrum, period, cone of influence, and significance levels."""
    return run_cwt_batch([cwt_data], normalize=normalize, standardize=standardize,
                         calculate_significance=calculate_significance,
                         significance_level=significance_level, **kwargs)[0]


def run_cwt_batch(cwt_data_list: List[DataForCWT], normalize: bool = True,
                  standardize: bool = False, calculate_significance: bool = True,
                  significance_level: float = 0.95, **kwargs) -> List[ResultsFromCWT]:
    """``run_cwt`` over many series (engine extension; the reference loops in
    src/utils/transform_helpers.py:116-123).  Series of one length and mother wavelet
    share one moments launch, one affine launch and ONE fused CWT launch; each keeps its
    own AR(1) significance (a [B, S] multiplier).  Results are those of run_cwt per series."""
    out: List[ResultsFromCWT] = [None] * len(cwt_data_list)
    groups: dict = {}
    for i, d in enumerate(cwt_data_list):
        groups.setdefault((np.asarray(d.y_values).size, kernel_mother(d.mother_wavelet)), []).append(i)
    for (n0, _), idx in groups.items():
        # any pycwt mother (Morlet, Paul, DOG / MexicanHat), as pycwt.cwt takes them
        mother = as_mother(cwt_data_list[idx[0]].mother_wavelet)
        y = transforms._to_dev(np.stack([np.asarray(cwt_data_list[i].y_values, dtype=np.float64)
                                         for i in idx]))
        mom_y = ops.series_moments(y)
        if standardize:
            # kwargs go to standardize_series as in the reference (:102): an unknown keyword
            # raises TypeError there and here
            coef = transforms.standardize_coefs(mom_y, **kwargs)
        else:  # quirk B.1: `normalize` has no effect
            coef = torch.zeros((len(idx), 3), dtype=torch.float64, device=y.device)
            coef[:, 2] = 1.0
        x32 = ops.affine(y, coef, torch.float32)
        m = transforms._np(mom_y)
        sj, freqs = transforms.scales_for(n0, DT, DJ, S0, J, mother)
        sig_scale = None
        if calculate_significance:
            rows = []
            for k in range(len(idx)):  # quirk B.2: AR(1) of y_values, not the standardised series
                alpha, _, _ = transforms._ar1_from_moments(m[k, 4], m[k, 5], int(m[k, 6]))
                signif, _ = transforms.significance(1.0, DT, sj, 0, alpha,
                                                    significance_level=significance_level,
                                                    wavelet=mother)
                rows.append(1.0 / signif)
            sig_scale = np.stack(rows)
        res = ops.cwt_morlet(x32, sj, DT, sig_scale=sig_scale, want_w=False, want_power=True,
                             want_sig=calculate_significance, mother=mother)
        power = transforms._np(res["power"], np.float64)
        sig = transforms._np(res["sig"], np.float64) if calculate_significance else None
        coi = transforms.cone_of_influence(n0, DT, mother)
        for k, i in enumerate(idx):
            out[i] = ResultsFromCWT(power[k], 1 / freqs, None if sig is None else sig[k], coi.copy())
    return out


def plot_cwt(cwt_ax, cwt_data: Type[DataForCWT], cwt_results: Type[ResultsFromCWT],
             include_significance: bool = True, include_cone_of_influence: bool = True,
             **kwargs) -> None:
    """Filled contours of log2 power over (time, log2 period) at log2(levels), the
    significance contour and the COI shading, period axis inverted with one tick per
    octave (src/cwt.py:138-185).  kwargs: ``cmap`` plus the helpers' keys."""
    log_period = np.log2(cwt_results.period)
    cwt_ax.contourf(cwt_data.time_range, log_period, np.log2(cwt_results.power),
                    np.log2(cwt_data.levels), extend="both", cmap=kwargs["cmap"])
    if include_significance:
        plot_signficance_levels(cwt_ax, cwt_results.significance_levels, cwt_data.time_range,
                                cwt_results.period, **kwargs)
    if include_cone_of_influence:
        plot_cone_of_influence(cwt_ax, cwt_results.coi, cwt_data.time_range, cwt_data.levels,
                               cwt_results.period, cwt_data.delta_t, tranform_type="cwt",
                               **kwargs)
    bottom, top = cwt_ax.get_ylim()
    cwt_ax.set_ylim(top, bottom)  # short periods at the top
    octave = 2 ** np.arange(np.ceil(np.log2(cwt_results.period.min())),
                            np.ceil(np.log2(cwt_results.period.max())))
    cwt_ax.set_yticks(np.log2(octave))
    cwt_ax.set_yticklabels(octave, size=15)
