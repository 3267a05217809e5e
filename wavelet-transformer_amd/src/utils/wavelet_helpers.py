"""Helper functions for wavelet transforms (reference: src/utils/wavelet_helpers.py).

``standardize_series`` runs on the GPU (moments + affine kernels, fp64).
``normalize_xwt_results`` and ``align_series`` are the reference's O(S)/O(n) host
glue on arrays the caller already holds; the engine's own ``run_xwt`` computes the
[S, n] power and ratio on the GPU and only uses the COI-polygon part on the host.
The two plot helpers draw on a caller-owned matplotlib ``Axes`` exactly the artists
the reference draws (one contour set at level 1, one filled COI polygon), so the
app's figures come out the same (src/utils/wavelet_helpers.py:81-153).
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


def normalize_xwt_results(signal_size: npt.NDArray, xwt_coeffs: npt.NDArray, coi: npt.NDArray,
                          coi_min: float, freqs: npt.NDArray, signif: npt.NDArray
                          ) -> tuple[npt.NDArray, npt.NDArray, npt.NDArray, npt.NDArray]:
    """(period, power = |W12|^2, sig95 = power / signif, coi polygon) (:60-78)."""
    period = 1 / freqs
    power = np.abs(xwt_coeffs) ** 2
    sig95 = power / (np.ones([1, signal_size]) * signif[:, None])
    return period, power, sig95, coi_polygon(coi, period, coi_min)


def plot_signficance_levels(ax, signficance_levels: npt.NDArray, t_values: npt.NDArray,
                            period: npt.NDArray, **kwargs) -> None:
    """Contour where the significance ratio crosses 1 (levels [-99, 1]) over
    (time, log2 period) (:81-101).  kwargs: ``sig_colors``, ``sig_linewidths``."""
    ax.contour(
        t_values,
        np.log2(period),
        signficance_levels,
        [-99, 1],
        colors=kwargs["sig_colors"],
        linewidths=kwargs["sig_linewidths"],
        extent=[t_values.min(), t_values.max(), 0, max(period)],
    )


def _coi_outline(t_values, dt):
    """Time axis of the COI polygon: the series' times, then two points one step past
    the end and two one step before the start (closing the shape along the bottom)."""
    after, before = t_values[-1:] + dt, t_values[:1] - dt
    return np.concatenate([t_values, after, after, before, before])


def plot_cone_of_influence(ax, coi: npt.NDArray, t_values: npt.NDArray, levels: list[float],
                           period: npt.NDArray, dt: float, tranform_type: str, **kwargs) -> None:
    """Shade the cone of influence (:104-153).  ``tranform_type`` "cwt" builds the
    polygon from the per-sample COI periods (log2, closed at ``levels[2]`` and the
    longest period, clipped below at -2.5); "xwt" takes ``coi`` as an already-built
    polygon (``normalize_xwt_results``).  kwargs: ``coi_color``, ``coi_alpha``,
    ``coi_hatch``."""
    if tranform_type == "cwt":
        longest = np.log2(period[-1:])
        y = np.concatenate([np.log2(coi), [levels[2]], longest, longest, [levels[2]]]).clip(min=-2.5)
    if tranform_type == "xwt":
        y = coi
    ax.fill(_coi_outline(t_values, dt), y, kwargs["coi_color"], alpha=kwargs["coi_alpha"],
            hatch=kwargs["coi_hatch"])
