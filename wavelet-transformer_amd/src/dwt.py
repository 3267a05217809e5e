"""Smoothing of signals via wavelet reconstruction (reference: src/dwt.py).

Pyramid DWT / inverse DWT (mode 'symmetric') run on the GPU (``wtmi_wavedec`` /
``wtmi_waverec``).  ``ResultsFromDWT.smooth_signal`` reconstructs all ``levels``
smoothed signals in ONE batched launch (one variant per level) instead of the
reference's loop of ``pywt.waverec`` calls (src/dwt.py:53-73).  Coefficient lists
keep pywt order ``[cA_J, cD_J, ..., cD_1]`` (quirk B.10).
"""

from __future__ import annotations

import hashlib
import logging
import threading
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Type

import numpy as np
import numpy.typing as npt

from wtmi import transforms
from wtmi.wavelets import Wavelet, as_filter_bank
from src.utils.wavelet_helpers import align_series

logger = logging.getLogger(__name__)

MOTHER = Wavelet("db4")


@dataclass
class DataForDWT:
    """Holds data for discrete wavelet transform"""

    y_values: npt.NDArray
    mother_wavelet: Type
    levels: int = None


@dataclass
class ResultsFromDWT:
    """`coeffs`: transform coefficients; `levels`: levels applied;
    `smoothed_signal_dict`: smoothed signal for each level"""

    coeffs: npt.NDArray
    levels: int
    smoothed_signal_dict: Dict[int, Dict[str, npt.NDArray]] = field(default_factory=dict)

    def smooth_signal(self, y_values: npt.NDArray, mother_wavelet: Type
                      ) -> Dict[int, Dict[str, npt.NDArray]]:
        """signal_dict[l]: reconstruction with the last l detail arrays zeroed."""
        nlist = len(self.coeffs)
        full = (1 << nlist) - 1
        lv = list(range(self.levels, 0, -1))
        masks = []
        for lvl in lv:
            m = full
            for k in range(1, lvl + 1):
                m &= ~(1 << (nlist - k))
            masks.append(m)
        recs = transforms.waverec_variants(self.coeffs, mother_wavelet, masks)
        signals_dict = {}
        for i, lvl in enumerate(lv):
            print(f"s_{lvl} stored with key {lvl}")  # reference prints too (quirk B.12)
            smooth_coeffs = [np.array(c, copy=True) for c in self.coeffs]
            for k in range(1, lvl + 1):
                smooth_coeffs[-k] = np.zeros_like(smooth_coeffs[-k])
            signals_dict[lvl] = {"coeffs": smooth_coeffs, "signal": trim_signal(y_values, recs[i])}
        self.smoothed_signal_dict = signals_dict


def trim_signal(original_signal: npt.NDArray, reconstructed: npt.NDArray) -> npt.NDArray:
    """Drop the FIRST reconstructed sample for odd-length inputs (quirk B.12)."""
    if len(original_signal) % 2 != 0:
        logger.warning("Trimming signal at beginning")
        return reconstructed[1:]
    return reconstructed


def run_dwt(dwt_data: Type[DataForDWT]) -> Type[ResultsFromDWT]:
    """Coefficients from a pyramid DWT; ``levels=None`` means pywt's maximum level."""
    return run_dwt_batch([dwt_data])[0]


def run_dwt_batch(dwt_data_list: List[DataForDWT]) -> List[ResultsFromDWT]:
    """``run_dwt`` over many series (engine extension; the reference loops in
    src/utils/transform_helpers.py:89-113): series of one length, wavelet and level share
    ONE analysis launch."""
    out = []
    for d, coeffs in zip(dwt_data_list, wavedec_batch(dwt_data_list)):
        if d.levels is None:
            dwt_levels = transforms.dwt_max_level(len(d.y_values),
                                                  as_filter_bank(d.mother_wavelet).dec_len)
            print(f"""Max decomposition level of {dwt_levels} for time series length
            of {len(d.y_values)}""")
        else:
            dwt_levels = d.levels
        out.append(ResultsFromDWT(coeffs, dwt_levels))
    return out


def wavedec_batch(dwt_data_list: List[DataForDWT]) -> list:
    """Coefficient lists of pywt.wavedec(y_values, mother_wavelet, level=levels) for each
    entry, one launch per group of equal (length, wavelet, level)."""
    out: list = [None] * len(dwt_data_list)
    groups: dict = {}
    for i, d in enumerate(dwt_data_list):
        w = as_filter_bank(d.mother_wavelet)
        groups.setdefault((len(d.y_values), w.name, tuple(w.dec_lo), d.levels), []).append(i)
    for (_, _, _, level), idx in groups.items():
        w = as_filter_bank(dwt_data_list[idx[0]].mother_wavelet)
        rows = np.stack([np.asarray(dwt_data_list[i].y_values, dtype=np.float64) for i in idx])
        for k, c in zip(idx, transforms.wavedec_batch(rows, w, level=level)):
            out[k] = c
    return out


class _ComponentCache:
    """All single-entry reconstructions of one coefficient list, from ONE batched launch.

    The reference's callers reconstruct the components of a list one level at a time
    (src/regression.py:113-114 alternates two lists over levels + 1 calls; src/dwt.py:123-156
    loops too): the first call for a list computes every component in one ``waverec`` launch
    (``n_variants`` = the list's length) and the others are served from here.  Keyed by the
    coefficients' content (and the wavelet), so a list mutated in place is a new key; a few
    lists are kept (least recently used dropped); thread-safe (Streamlit sessions share the
    module)."""

    def __init__(self, size: int = 8):
        self.size = size
        self._d: "OrderedDict[tuple, list]" = OrderedDict()
        self._lock = threading.Lock()

    @staticmethod
    def key(coeffs: list, wavelet) -> tuple:
        h = hashlib.blake2b(digest_size=16)
        for c in coeffs:
            a = np.ascontiguousarray(c)
            h.update(str((a.dtype.str, a.shape)).encode())
            h.update(a.tobytes())
        w = as_filter_bank(wavelet)
        return (h.hexdigest(), w.name, tuple(w.dec_lo))

    def get(self, coeffs: list, wavelet, level: int):
        k = self.key(coeffs, wavelet)
        with self._lock:
            parts = self._d.get(k)
            if parts is not None:
                self._d.move_to_end(k)
        if parts is None:
            parts = transforms.waverec_variants(coeffs, wavelet, [1 << j for j in range(len(coeffs))])
            with self._lock:
                self._d[k] = parts
                self._d.move_to_end(k)
                while len(self._d) > self.size:
                    self._d.popitem(last=False)
        return np.array(parts[level], copy=True)


_COMPONENTS = _ComponentCache()


def reconstruct_signal_component(signal_coeffs: list, wavelet: str, level: int):
    """Inverse DWT keeping only list entry ``level`` (src/dwt.py:110-120); every component
    of the list comes from one batched launch on the first call (``_ComponentCache``)."""
    if not 0 <= level < len(signal_coeffs):  # the reference zeroes every entry then
        return transforms.waverec_variants(signal_coeffs, wavelet, [0])[0]
    return _COMPONENTS.get(signal_coeffs, wavelet, level)


def _subplots(nrows, **kwargs):
    import matplotlib.pyplot as plt  # plotting only; the transforms never import matplotlib
    return plt.subplots(nrows, 1, **kwargs)


def plot_components(label: str, coeffs: npt.NDArray, time: npt.NDArray, levels: int,
                    wavelet: str, **kwargs):
    """One panel per component: the smooth S_J on top, then D_J .. D_1, each trimmed
    to the time axis (src/dwt.py:123-156).  All levels+1 single-entry reconstructions
    come from ONE batched inverse-DWT launch."""
    import matplotlib.pyplot as plt
    fig, ax = _subplots(levels + 1, **kwargs)
    parts = transforms.waverec_variants(coeffs, wavelet, [1 << lvl for lvl in range(levels + 1)])
    logger.warning("lengths x: %s, t: %s", len(parts[0]), len(time))
    for lvl in range(levels + 1):
        y = parts[lvl]
        if len(y) != len(time):
            y = align_series(time, y)
        ax[lvl].plot(time, y, label=label)
        title = rf"$S_{{{levels}}}$" if lvl == 0 else rf"$D_{{{levels + 1 - lvl}}}$"
        ax[lvl].set_title(title, size=15)
    plt.legend(loc="upper left")
    return fig


def plot_smoothing(smooth_signals: dict, original_t: npt.NDArray, original_y: npt.NDArray,
                   ascending: bool = False, **kwargs):
    """One panel per smoothed signal over the original (src/dwt.py:159-184); panel
    order follows the dict, reversed when ``ascending``."""
    fig, axs = _subplots(len(smooth_signals), **kwargs)
    items = list(smooth_signals.items())
    if ascending:
        items = items[::-1]
    for panel, (level, signal) in enumerate(items):
        axs[panel].plot(original_t, original_y, label="Original")
        axs[panel].plot(original_t, signal["signal"])
        axs[panel].set_title(rf"Approximation: $S_{{j-{len(smooth_signals) - level}}}$", size=15)
        if panel == 0:
            axs[panel].legend(loc="upper right")
        else:
            axs[panel].legend("", frameon=False)
    return fig
