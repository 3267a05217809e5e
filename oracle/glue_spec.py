"""CPU restatement of the reference wrapper glue around pycwt / pywt.

TEST INFRASTRUCTURE ONLY (see ``oracle/pycwt_spec.py`` header for the rules).

Restates, line for line in behaviour (not in text):
  * ``standardize_series``      src/utils/wavelet_helpers.py:22-57
  * ``normalize_xwt_results``   src/utils/wavelet_helpers.py:60-78
  * ``run_cwt``                 src/cwt.py:85-135  (incl. quirks B.1-B.3)
  * ``run_xwt``                 src/xwt.py:83-139  (incl. quirk B.5: phase at dj=1/12)
  * ``run_wct``                 src/wct.py:96-140  (sig=False path)
  * ``calculate_phase_difference`` src/xwt.py:142-154, src/wct.py:143-158
  * ``ResultsFromDWT.smooth_signal`` / ``reconstruct_signal_component`` /
    ``trim_signal``             src/dwt.py:53-120
"""

from __future__ import annotations

import numpy as np

from . import pycwt_spec as pc
from . import dwt_spec

CWT_DT = 1 / 12
CWT_DJ = 1 / 12
CWT_S0 = 2 * CWT_DT
CWT_J = 7 / CWT_DJ


def standardize_series(series, detrend=True, standardize=True, remove_mean=False):
    series = np.asarray(series)
    std = series.std()
    smean = series.mean()
    if detrend and remove_mean:
        raise ValueError("Only standardize by either removing secular trend or mean, not both.")
    if detrend:
        xs = np.arange(0, series.size)
        p = np.polyfit(xs, series, 1)
        snorm = series - np.polyval(p, xs)
    else:
        snorm = series
    if remove_mean:
        snorm = snorm - smean
    if standardize:
        snorm = snorm / std
    return snorm


def normalize_xwt_results(signal_size, xwt_coeffs, coi, coi_min, freqs, signif):
    period = 1 / freqs
    power = np.abs(xwt_coeffs) ** 2
    sig95 = power / (np.ones([1, signal_size]) * signif[:, None])
    coi_plot = np.concatenate(
        [np.log2(coi), [1e-9], np.log2(period[-1:]), np.log2(period[-1:]), [1e-9]]
    ).clip(min=coi_min)
    return period, power, sig95, coi_plot


def phase_uv(phase):
    angle = 0.5 * np.pi - phase
    return np.cos(angle), np.sin(angle)


def run_cwt(y_values, n_obs, mother=None, normalize=True, standardize=False,
            calculate_significance=True, significance_level=0.95,
            dt=CWT_DT, dj=CWT_DJ, s0=CWT_S0, J=CWT_J, **kwargs):
    """Returns (power, period, sig_ratio_or_None, coi)."""
    mother = mother or pc.Morlet(6)
    y = np.asarray(y_values)
    if standardize:
        dat = standardize_series(y, **kwargs)
    else:
        dat = y  # quirk B.1: normalize=True is a no-op
    alpha, _, _ = pc.ar1(y)  # quirk B.2: AR(1) on y_values, not dat
    wave, scales, freqs, coi, _, _ = pc.cwt(dat, dt, dj, s0, J, mother)
    power = np.abs(wave) ** 2
    period = 1 / freqs
    sig = None
    if calculate_significance:
        signif, _ = pc.significance(1.0, dt, scales, 0, alpha,
                                    significance_level=significance_level, wavelet=mother)
        sig = power / (np.ones([1, n_obs]) * signif[:, None])
    return power, period, sig, coi


def run_xwt(y1, y2, dt, dj, s0, levels, mother=None):
    """Returns (power, period, sig95, coi_plot, u, v)."""
    mother = mother or pc.Morlet(6)
    W12, coi, freqs, signif = pc.xwt(y1, y2, dt=dt, dj=dj, s0=s0, wavelet=mother)
    period, power, sig95, coi_plot = normalize_xwt_results(
        np.asarray(y1).size, W12, coi, np.log2(levels[2]), freqs, signif)
    # quirk B.5: ``delta_j=`` is swallowed by **kwargs -> dj defaults to 1/12
    _, phase, _, _, _ = pc.wct(y1, y2, dt, delta_j=dj, s0=s0, J=-1, sig=False,
                              wavelet=mother, normalize=True, cache=True)
    u, v = phase_uv(phase)
    return power, period, sig95, coi_plot, u, v


def run_wct(y1, y2, dt, dj, s0, mother=None):
    """sig=False path. Returns (coherence, period, sig95, coi, u, v)."""
    mother = mother or pc.Morlet(6)
    coh, phase, coi, freqs, signif = pc.wct(y1, y2, dt, dj=dj, s0=s0, J=-1, sig=False,
                                            wavelet=mother, normalize=True, cache=True)
    period = 1 / freqs
    n = np.asarray(y1).size
    with np.errstate(divide="ignore", invalid="ignore"):
        sig95 = np.abs(coh) / (np.ones([1, n]) * signif[:, None])  # quirk B.8 -> inf
    u, v = phase_uv(phase)
    return coh, period, sig95, coi, u, v


def trim_signal(original, reconstructed):
    if len(original) % 2 != 0:
        return reconstructed[1:]
    return reconstructed


def dwt_smooth_signal(coeffs, levels, y_values, rec_lo, rec_hi):
    out = {}
    for lvl in range(levels, 0, -1):
        c = [np.array(a, copy=True) for a in coeffs]
        for k in range(1, lvl + 1):
            c[-k] = np.zeros_like(c[-k])
        rec = dwt_spec.waverec(c, rec_lo, rec_hi)
        out[lvl] = {"coeffs": c, "signal": trim_signal(y_values, rec)}
    return out


def reconstruct_signal_component(coeffs, level, rec_lo, rec_hi):
    c = [np.array(a) if i == level else np.zeros_like(a) for i, a in enumerate(coeffs)]
    return dwt_spec.waverec(c, rec_lo, rec_hi)
