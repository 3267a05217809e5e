"""Helper functions for wavelet transforms (reference: src/utils/wavelet_helpers.py).

``standardize_series`` runs on the GPU (moments + affine kernels, fp64).
``normalize_xwt_results`` and ``align_series`` are the reference's O(S)/O(n) host
glue on arrays the caller already holds; the engine's own ``run_xwt`` computes the
[S, n] power and ratio on the GPU and only uses the COI-polygon part on the host.
"""

from __future__ import annotations

import logging

import numpy as np
import numpy.typing as npt

from wtmi import transforms

logger = logging.getLogger(__name__)


def align_series(t_values: npt.NDArray, series_vlaues: npt.NDArray) -> npt.NDArray:
    """Trim the leading samples of a series longer than its time axis (:13-19)."""
    if len(series_vlaues) != len(t_values):
        logger.warning("Trimming series signal")
        difference = np.abs(len(series_vlaues) - len(t_values))
        return series_vlaues[difference:]
    return series_vlaues


def standardize_series(series: npt.NDArray, detrend: bool = True, standardize: bool = True,
                       remove_mean: bool = False) -> npt.NDArray:
    """Detrend (least-squares line) or demean, then divide by the ORIGINAL std (:22-57).
    Raises ValueError when both detrend and remove_mean are requested."""
    return transforms.standardize_series(series, detrend=detrend, standardize=standardize,
                                         remove_mean=remove_mean)


def coi_polygon(coi: npt.NDArray, period: npt.NDArray, coi_min: float) -> npt.NDArray:
    """XWT cone-of-influence polygon in log2 space, clipped at coi_min (:73-77)."""
    return np.concatenate(
        [np.log2(coi), [1e-9], np.log2(period[-1:]), np.log2(period[-1:]), [1e-9]]
    ).clip(min=coi_min)


def normalize_xwt_results(signal_size, xwt_coeffs, coi, coi_min, freqs, signif):
    """(period, power = |W12|^2, sig95 = power / signif, coi polygon) (:60-78)."""
    period = 1 / freqs
    power = np.abs(xwt_coeffs) ** 2
    sig95 = power / (np.ones([1, signal_size]) * signif[:, None])
    return period, power, sig95, coi_polygon(coi, period, coi_min)
