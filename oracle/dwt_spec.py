"""CPU restatement of the pyramid DWT the reference calls through PyWavelets.

TEST INFRASTRUCTURE ONLY (see ``oracle/pycwt_spec.py`` header for the rules).

The reference calls ``pywt.wavedec`` / ``pywt.waverec`` / ``pywt.dwt_max_level``
(PyWavelets 1.9.0, ``requirements.txt:39``) from ``src/dwt.py:95,104,120`` and
``src/utils/transform_helpers.py:41,96``, always with the default mode
``"symmetric"`` (half-sample symmetric extension).

Pinning: ``tests/golden/dwt_golden.npz`` holds outputs of PyWavelets 1.1.1 (the
copy importable in this container under ``/opt/conda/bin/python3.9``), generated
by ``tests/golden/make_golden.py``; the symmetric-mode arithmetic is unchanged
between 1.1.1 and 1.9.0.

Conventions restated here (checked against pywt in ``tests/test_oracle_dwt.py``):

* analysis:  ``c[i] = sum_{j<F} f[j] * xe[2i + 1 - j]``, ``i < (n + F - 1)//2``,
  with ``xe`` the half-sample-symmetric extension of ``x``;
* synthesis: ``y[m] = sum_i cA[i] rec_lo[m + F - 2 - 2i] + cD[i] rec_hi[...]``,
  ``m < 2*len(cA) - F + 2``;
* ``waverec`` trims ``a`` to ``len(d)`` when it is one longer.
"""

from __future__ import annotations

import numpy as np


def symmetric_index(idx, n):
    """Map any integer index onto [0, n) by repeated half-sample reflection."""
    idx = np.asarray(idx, dtype=np.int64)
    period = 2 * n
    m = np.mod(idx, period)
    return np.where(m < n, m, period - 1 - m)


def dwt_max_level(data_len: int, filter_len: int) -> int:
    if filter_len < 2:
        raise ValueError("invalid wavelet filter length")
    if data_len < filter_len - 1:
        return 0
    return int(np.floor(np.log2(data_len / (filter_len - 1))))


def dwt(x, dec_lo, dec_hi):
    x = np.asarray(x, dtype=np.float64)
    F = len(dec_lo)
    n = x.size
    M = (n + F - 1) // 2
    i = np.arange(M)[:, None]
    j = np.arange(F)[None, :]
    xe = x[symmetric_index(2 * i + 1 - j, n)]
    return xe @ np.asarray(dec_lo, float), xe @ np.asarray(dec_hi, float)


def idwt(cA, cD, rec_lo, rec_hi):
    cA = np.asarray(cA, dtype=np.float64)
    cD = np.asarray(cD, dtype=np.float64)
    F = len(rec_lo)
    M = cA.size
    L = 2 * M - F + 2
    y = np.zeros(L)
    rec_lo = np.asarray(rec_lo, float)
    rec_hi = np.asarray(rec_hi, float)
    for i in range(M):
        # coefficient i touches outputs m with 0 <= m + F - 2 - 2i < F
        m0 = 2 * i - F + 2
        ks = np.arange(F)
        ms = m0 + ks
        ok = (ms >= 0) & (ms < L)
        y[ms[ok]] += cA[i] * rec_lo[ks[ok]] + cD[i] * rec_hi[ks[ok]]
    return y


def wavedec(x, dec_lo, dec_hi, level=None):
    """``[cA_J, cD_J, ..., cD_1]`` (pywt order)."""
    x = np.asarray(x, dtype=np.float64)
    F = len(dec_lo)
    if level is None:
        level = dwt_max_level(x.size, F)
    if level < 0:
        raise ValueError("Level value of %d is too low . Minimum level is 0." % level)
    out = []
    a = x
    for _ in range(level):
        a, d = dwt(a, dec_lo, dec_hi)
        out.append(d)
    out.append(a)
    out.reverse()
    return out


def waverec(coeffs, rec_lo, rec_hi):
    a, ds = coeffs[0], coeffs[1:]
    a = np.asarray(a, dtype=np.float64)
    for d in ds:
        d = np.asarray(d, dtype=np.float64)
        if a.size == d.size + 1:
            a = a[: d.size]
        elif a.size != d.size:
            raise ValueError("coefficient shape mismatch")
        a = idwt(a, d, rec_lo, rec_hi)
    return a
