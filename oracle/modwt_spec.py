"""CPU restatement of the reference MODWT (``src/modwt.py``).

TEST INFRASTRUCTURE ONLY (see ``oracle/pycwt_spec.py`` header for the rules).

Pinning: golden vectors in ``tests/golden/modwt_golden.npz`` were produced by
running the reference's OWN functions (``src/modwt.py:56-251``, extracted by AST
from ``/root/reference`` in the build container, see
``tests/golden/make_golden.py``); ``tests/test_oracle_modwt.py`` checks this
restatement against them.

Two forms are provided:

* ``modwt`` / ``imodwt`` use the same algorithm as the reference -- zero-stuffed
  dilated kernels filtered with ``scipy.ndimage.convolve1d(mode="wrap")``
  (``src/modwt.py:86-123``), so the CPU-baseline cost is the reference's cost
  (work proportional to 8*2**(j-1) taps per sample at level j).
* ``modwt_direct`` / ``imodwt_direct`` are the textbook Percival-Walden sums
  ``W_j[t] = sum_l h_l V_{j-1}[(t - 2**(j-1) l) mod N]`` used to cross-check.
"""

from __future__ import annotations

import numpy as np
from scipy.ndimage import convolve1d

SQRT2 = np.sqrt(2.0)


def _stuffed(taps, j):
    d = 2 ** (j - 1)
    ker = np.zeros(len(taps) * d)
    ker[::d] = taps
    return ker


def analysis_level(taps_t, v_prev, j):
    """One pyramid-free analysis step; cf. ``circular_convolve_d`` (src/modwt.py:86-102)."""
    ker = _stuffed(taps_t, j)
    return convolve1d(v_prev, ker, mode="wrap", origin=-len(ker) // 2)


def synthesis_level(h_t, g_t, w_j, v_j, j):
    """One synthesis step; cf. ``circular_convolve_s`` (src/modwt.py:105-123)."""
    hk = _stuffed(h_t, j)[::-1]
    gk = _stuffed(g_t, j)[::-1]
    out = convolve1d(w_j, hk, mode="wrap", origin=(len(hk) - 1) // 2)
    out += convolve1d(v_j, gk, mode="wrap", origin=(len(gk) - 1) // 2)
    return out


def modwt(x, dec_lo, dec_hi, level):
    """Rows ``[W_1 .. W_J, V_J]`` (src/modwt.py:126-144). Output dtype follows x."""
    h_t = np.asarray(dec_hi, dtype=np.float64) / SQRT2
    g_t = np.asarray(dec_lo, dtype=np.float64) / SQRT2
    rows = []
    v = x
    for j in range(1, level + 1):
        rows.append(analysis_level(h_t, v, j))
        v = analysis_level(g_t, v, j)
    rows.append(v)
    return np.vstack(rows)


def imodwt(w, dec_lo, dec_hi):
    """Inverse MODWT (src/modwt.py:147-160)."""
    h_t = np.asarray(dec_hi, dtype=np.float64) / SQRT2
    g_t = np.asarray(dec_lo, dtype=np.float64) / SQRT2
    level = len(w) - 1
    v = w[-1]
    for j in range(level, 0, -1):
        v = synthesis_level(h_t, g_t, w[j - 1], v, j)
    return v


def modwt_direct(x, dec_lo, dec_hi, level):
    x = np.asarray(x, dtype=np.float64)
    h_t = np.asarray(dec_hi, dtype=np.float64) / SQRT2
    g_t = np.asarray(dec_lo, dtype=np.float64) / SQRT2
    N = x.size
    t = np.arange(N)
    v = x
    rows = []
    for j in range(1, level + 1):
        d = 2 ** (j - 1)
        w = sum(h_t[l] * v[(t - d * l) % N] for l in range(len(h_t)))
        v = sum(g_t[l] * v[(t - d * l) % N] for l in range(len(g_t)))
        rows.append(w)
    rows.append(v)
    return np.vstack(rows)


def imodwt_direct(w, dec_lo, dec_hi):
    w = np.asarray(w, dtype=np.float64)
    h_t = np.asarray(dec_hi, dtype=np.float64) / SQRT2
    g_t = np.asarray(dec_lo, dtype=np.float64) / SQRT2
    level = w.shape[0] - 1
    N = w.shape[1]
    t = np.arange(N)
    v = w[-1]
    for j in range(level, 0, -1):
        d = 2 ** (j - 1)
        v = sum(
            h_t[l] * w[j - 1][(t + d * l) % N] + g_t[l] * v[(t + d * l) % N]
            for l in range(len(h_t))
        )
    return v


def modwtmra(w, dec_lo, dec_hi):
    """MRA rows ``[D_1 .. D_J, S_J]``; row j equals the inverse MODWT of the
    isolated row j (reference ``modwtmra`` src/modwt.py:163-194 builds the same
    operator from dense equivalent filters; probe C.8b)."""
    w = np.asarray(w)
    out = []
    for j in range(w.shape[0]):
        iso = np.zeros_like(w)
        iso[j] = w[j]
        out.append(imodwt(iso, dec_lo, dec_hi))
    return np.vstack(out)


def smooth_signal(modwt_coeffs, dec_lo, dec_hi, levels):
    """``src/modwt.py:232-251``: key l -> rows 0..l-1 zeroed, then inverse."""
    out = {}
    for lvl in range(levels, 0, -1):
        c = np.array(modwt_coeffs, copy=True)
        c[:lvl] = 0
        out[lvl] = {"coeffs": c, "signal": imodwt(c, dec_lo, dec_hi)}
    return out
