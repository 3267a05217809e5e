"""Maximal-overlap DWT (reference: src/modwt.py:56-285).

``modwt`` / ``imodwt`` run the a-trous cascades on the GPU (``wtmi_modwt`` /
``wtmi_imodwt``: one workgroup per series, all J levels LDS-resident, only the L
non-zero taps per level).  ``modwtmra`` and ``smooth_signal`` are masked inverse
transforms (row j of the MRA = inverse of the isolated row j, probe C.8b).
Row order is the reference's ``[W_1 .. W_J, V_J]``; output dtype follows the input
dtype (float32 in -> float32 out, quirk B.11).

The reference module also exports its single-level helpers (``upArrow_op``,
``period_list``, ``circular_convolve_{d,s,mra}``), the per-component OLS
``time_scale_regression`` and ``plot_smoothing``.  They are re-provided with the same
signatures and results for code that imports them; none of them is on the transform
path (the GPU cascades never call them).  The circular convolutions are written as
periodic index sums (Percival & Walden's form) on the host.
"""

from __future__ import annotations

import numpy as np
import numpy.typing as npt

from wtmi import transforms
from wtmi.wavelets import Wavelet

MOTHER = Wavelet("db4")


def modwt(x, filters, level):
    """filters: 'db1', 'db2', 'haar', ... (or a filter-bank object); returns [level+1, N]."""
    return transforms.modwt(x, filters, level)


def imodwt(w, filters):
    """Inverse MODWT of rows [W_1 .. W_J, V_J]."""
    return transforms.imodwt(w, filters)


def modwtmra(w, filters):
    """Multiresolution analysis [D_1 .. D_J, S_J]."""
    w = np.asarray(w)
    return np.vstack([transforms.imodwt(w, filters, keep_mask=1 << j) for j in range(w.shape[0])])


def smooth_signal(modwt_coeffs: npt.NDArray, mother_wavelet: str, levels: int
                  ) -> dict[int, dict[str, npt.NDArray]]:
    """signal_dict[l]: inverse with detail rows 0..l-1 zeroed (src/modwt.py:232-251)."""
    signals_dict = {}
    c = np.asarray(modwt_coeffs)
    full = (1 << c.shape[0]) - 1
    for lvl in range(levels, 0, -1):
        print(f"s_{lvl} stored with key {lvl}")
        smooth_coeffs = c.copy()
        smooth_coeffs[:lvl] = 0
        keep = full & ~((1 << lvl) - 1)
        signals_dict[lvl] = {"coeffs": smooth_coeffs,
                             "signal": transforms.imodwt(c, mother_wavelet, keep_mask=keep)}
    return signals_dict


# --------------------------------------------------- the reference's host-side helpers
def upArrow_op(li, j):
    """Filter ``li`` upsampled for level j: 2**(j-1) - 1 zeros between taps; [1] at j = 0
    (src/modwt.py:56-63)."""
    if j == 0:
        return [1]
    step = 2 ** (j - 1)
    out = np.zeros(step * (len(li) - 1) + 1)
    out[::step] = li
    return out


def period_list(li, N):
    """Periodise a filter to length N by summing its N-blocks (src/modwt.py:66-78).  A
    filter shorter than N comes back zero-padded to N (as a plain array)."""
    li = list(li)
    padded = np.array(li + [0] * (N - len(li) % N))
    if padded.size < 2 * N:
        return padded
    return padded.reshape(-1, N).sum(axis=0)


def _taps(h, d, n, sign):
    """Periodic gather positions (t + sign * d * l) mod n for every tap l."""
    t = np.arange(n)[None, :]
    return (t + sign * d * np.arange(len(h))[:, None]) % n


def circular_convolve_mra(h_j_o, w_j):
    """D_j[t] = sum_k h_j_o[k] w_j[(t + k) mod N] (src/modwt.py:81-83)."""
    h = np.asarray(h_j_o, dtype=np.float64)
    w = np.asarray(w_j)
    out = np.einsum("k,kt->t", h, w[_taps(h, 1, w.size, +1)])
    return out.astype(w.dtype) if w.dtype in (np.float32, np.float64) else out


def circular_convolve_d(h_t, v_j_1, j):
    """Level-j analysis: w_j[t] = sum_l h_t[l] v_{j-1}[(t - 2**(j-1) l) mod N]
    (src/modwt.py:86-102)."""
    h = np.asarray(h_t, dtype=np.float64)
    v = np.asarray(v_j_1)
    out = np.einsum("l,lt->t", h, v[_taps(h, 2 ** (j - 1), v.size, -1)])
    return out.astype(v.dtype) if v.dtype in (np.float32, np.float64) else out


def circular_convolve_s(h_t, g_t, w_j, v_j, j):
    """Level-j synthesis: v_{j-1}[t] = sum_l h_t[l] w_j[(t + 2**(j-1) l) mod N]
    + g_t[l] v_j[(t + 2**(j-1) l) mod N] (src/modwt.py:105-123)."""
    h = np.asarray(h_t, dtype=np.float64)
    g = np.asarray(g_t, dtype=np.float64)
    w, v = np.asarray(w_j), np.asarray(v_j)
    idx = _taps(h, 2 ** (j - 1), v.size, +1)
    out = np.einsum("l,lt->t", h, w[idx]) + np.einsum("l,lt->t", g, v[idx])
    return out.astype(v.dtype) if v.dtype in (np.float32, np.float64) else out


def time_scale_regression(input_coeffs: npt.NDArray, output_coeffs: npt.NDArray, levels: int,
                          add_constant: bool = True):
    """OLS of output on input for each component S_J, D_J, ..., D_1, summarised side by
    side (src/modwt.py:197-229).  Needs statsmodels, as the reference does."""
    import statsmodels.api as sm
    from statsmodels.iolib.summary2 import summary_col
    fits = {}
    for j in range(levels + 1):
        name = f"S_{levels}" if j == 0 else f"D_{levels - j + 1}"
        print(f"Regressing on component vector {name}")
        x = sm.add_constant(input_coeffs[j]) if add_constant else input_coeffs[j]
        fits[name] = sm.OLS(output_coeffs[j], x).fit()
    return summary_col(list(fits.values()), stars=True, model_names=list(fits))


def plot_smoothing(smooth_signals: dict, original_t: npt.NDArray, original_y: npt.NDArray,
                   ascending: bool = False, **kwargs):
    """One panel per smoothed signal over the original (src/modwt.py:254-283)."""
    from src.dwt import plot_smoothing as _dwt_plot_smoothing
    return _dwt_plot_smoothing(smooth_signals, original_t, original_y, ascending=ascending,
                               **kwargs)
