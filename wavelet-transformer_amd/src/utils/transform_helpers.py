"""Helper functions to organize results of transforms (reference:
src/utils/transform_helpers.py).

Same dict builders as the reference (:21-135) -- the app's only batch API -- but the
``create_*_results_dict`` functions hand ALL requested series to the engine at once:
``cwt.run_cwt_batch`` / ``xwt.run_xwt_batch`` / ``dwt.run_dwt_batch`` issue one launch per
group of equal-length series instead of one Python-loop iteration (and one set of
launches) per series.  ``constants`` (ids, results_configs) is the app's own package and
is imported where the reference uses it, at call time, so this module imports without
the app tree.
"""

from __future__ import annotations

import logging

import pandas as pd

from src import cwt, dwt, xwt
from src.cwt import DataForCWT, ResultsFromCWT
from src.dwt import DataForDWT, ResultsFromDWT
from src.utils import wavelet_helpers
from src.xwt import DataForXWT, ResultsFromXWT
from wtmi import transforms

logger = logging.getLogger(__name__)


def create_dwt_dict(data_for_dwt: pd.DataFrame, measures_list: list[str], **kwargs
                    ) -> dict[str, DataForDWT]:
    """One DataForDWT per measure at pywt's maximum level for its length (:21-46)."""
    mother_wavelet = kwargs.get("mother_wavelet", dwt.MOTHER)
    out = {}
    for measure in measures_list:
        y_values = data_for_dwt[measure].to_numpy()
        level = transforms.dwt_max_level(len(y_values), mother_wavelet.dec_len)
        out[measure] = dwt.DataForDWT(y_values=y_values, mother_wavelet=mother_wavelet, levels=level)
    return out


def create_cwt_dict(data_for_cwt: pd.DataFrame, measures_list: list[str], **kwargs
                    ) -> dict[str, DataForCWT]:
    """One DataForCWT per measure over its non-missing dates, standardised (:49-63)."""
    from constants import ids
    out = {}
    for measure in measures_list:
        present = data_for_cwt[data_for_cwt[measure].notna()]
        y_values = wavelet_helpers.standardize_series(present[measure].to_numpy())
        out[measure] = cwt.DataForCWT(t_values=present[ids.DATE].to_numpy(), y_values=y_values,
                                      **kwargs)
    return out


def create_xwt_dict(data_for_xwt: pd.DataFrame, xwt_list: list[tuple[str, str]], **kwargs
                    ) -> dict[tuple[str, str], DataForXWT]:
    """One DataForXWT per pair over the rows where every column is present (:66-86)."""
    from constants import results_configs as rc
    out = {}
    complete = data_for_xwt.dropna()
    for comparison in xwt_list:
        y1 = wavelet_helpers.standardize_series(complete[comparison[0]].to_numpy(), **kwargs)
        y2 = wavelet_helpers.standardize_series(complete[comparison[1]].to_numpy(), **kwargs)
        out[comparison] = xwt.DataForXWT(
            y1_values=y1, y2_values=y2, mother_wavelet=rc.XWT_MOTHER_DICT[rc.XWT_MOTHER],
            delta_t=rc.XWT_DT, delta_j=rc.XWT_DJ, initial_scale=rc.XWT_S0, levels=rc.LEVELS)
    return out


def create_dwt_results_dict(dwt_data_dict: dict[str, DataForDWT], measures_list: list[str],
                            **kwargs) -> dict[str, ResultsFromDWT]:
    """Coefficients only, levels as given (:89-103): one batched analysis launch per
    group of equal-length series."""
    coeffs = dwt.wavedec_batch([dwt_data_dict[m] for m in measures_list])
    # the reference builds ResultsFromDWT(coeffs, data.levels) directly (no max-level fill-in)
    return {m: dwt.ResultsFromDWT(c, dwt_data_dict[m].levels) for m, c in zip(measures_list, coeffs)}


def create_dwt_regression_dict(dwt_data_dict: dict[str, DataForDWT], measures_list: list[str],
                               **kwargs) -> dict[str, ResultsFromDWT]:
    """run_dwt per measure (:106-113), batched."""
    if kwargs:  # the reference forwards them to run_dwt, which takes none
        raise TypeError(f"run_dwt() got unexpected keyword arguments {sorted(kwargs)}")
    return dict(zip(measures_list, dwt.run_dwt_batch([dwt_data_dict[m] for m in measures_list])))


def create_cwt_results_dict(cwt_data_dict: dict[str, DataForCWT], measures_list: list[str],
                            **kwargs) -> dict[str, ResultsFromCWT]:
    """run_cwt per measure (:116-123), batched: one CWT launch per length group."""
    return dict(zip(measures_list, cwt.run_cwt_batch([cwt_data_dict[m] for m in measures_list],
                                                     **kwargs)))


def create_xwt_results_dict(xwt_data_dict: dict[str, DataForXWT], xwt_list: list[tuple[str, str]],
                            **kwargs) -> ResultsFromXWT:
    """run_xwt per pair (:126-135), batched: one XWT launch (+ one phase launch) per group.
    Fails as run_xwt(data, **kwargs) does in the reference: unknown keywords raise TypeError,
    normalize=False NameError, a non-Morlet mother AttributeError -- at the first pair, after
    its lookup (KeyError first); with no pairs the reference's loop never runs: {}."""
    if not xwt_list:
        return {}
    xwt_data_dict[xwt_list[0]]
    unknown = sorted(set(kwargs) - {"normalize"})
    if unknown:
        raise TypeError(f"run_xwt() got unexpected keyword arguments {unknown}")
    if not kwargs.get("normalize", True):
        raise NameError("name 'signal_size' is not defined")
    return dict(zip(xwt_list, xwt.run_xwt_batch([xwt_data_dict[c] for c in xwt_list])))
