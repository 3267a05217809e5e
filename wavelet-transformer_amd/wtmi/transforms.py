"""pycwt / PyWavelets-shaped transforms on the MI355X engine (NumPy in, NumPy out).

These are the functions the reference's wrapper modules call on third-party
libraries -- ``pycwt.cwt / xwt / wct / ar1 / significance`` and ``pywt.wavedec /
waverec / dwt_max_level`` -- re-provided over the HIP kernels in ``ops``.  Every
[scales x time] array is produced on the GPU; the host only evaluates O(S) / O(n)
closed forms (scales, periods, cone of influence, AR(1) spectra) exactly as the
reference's libraries do.  Without a GPU every entry point raises.

Batched device-tensor variants (``*_batch``) take ``[batch, n]`` torch tensors and
return device tensors; the single-series functions wrap them.
"""

from __future__ import annotations

import math
import os
import threading
from typing import Optional

import numpy as np
import torch

from . import ops
from .wavelets import Morlet, as_filter_bank, as_morlet, as_mother


def device() -> torch.device:
    """The GPU the NumPy-facing functions run on (current HIP device)."""
    if not torch.cuda.is_available():
        raise RuntimeError("wtmi needs an MI355X GPU (torch.cuda.is_available() is False); "
                           "there is no CPU implementation")
    return torch.device("cuda", torch.cuda.current_device())


def _to_dev(y, dtype=torch.float64) -> torch.Tensor:
    if isinstance(y, torch.Tensor):
        return y.to(device=device() if not y.is_cuda else y.device, dtype=dtype)
    return torch.as_tensor(np.asarray(y), device=device()).to(dtype)


def _np(t: torch.Tensor, dtype=None) -> np.ndarray:
    a = t.detach().cpu().numpy()
    return a.astype(dtype, copy=False) if dtype is not None else a


# ------------------------------------------------------------------ closed forms
def scales_for(n0: int, dt: float, dj: float, s0: float, J: float, wavelet: Morlet):
    """pycwt ``cwt`` default resolution: s0 = 2 dt / lambda, J = round(log2(n0 dt / s0) / dj)."""
    if s0 == -1:
        s0 = 2 * dt / wavelet.flambda()
    if J == -1:
        J = int(np.round(np.log2(n0 * dt / s0) / dj))
    sj = s0 * 2 ** (np.arange(0, J + 1) * dj)
    freqs = 1 / (wavelet.flambda() * sj)
    return sj, freqs


def cone_of_influence(n0: int, dt: float, wavelet: Morlet) -> np.ndarray:
    coi = n0 / 2 - np.abs(np.arange(0, n0) - (n0 - 1) / 2)
    return wavelet.flambda() * wavelet.coi() * dt * coi


def chi2_ppf_dof2(p: float) -> float:
    """chi2.ppf(p, 2) = -2 ln(1 - p) (the only dof the Morlet path uses: dofmin = 2)."""
    return -2.0 * math.log1p(-p)


def _chi2_ppf(p: float, dof: int) -> float:
    if dof == 2:
        return chi2_ppf_dof2(p)
    from scipy.stats import chi2  # only for non-Morlet dofs
    return float(chi2.ppf(p, dof))


def ar1_spectrum(freqs, ar1=0.0):
    freqs = np.asarray(freqs)
    return (1 - ar1 ** 2) / np.abs(1 - ar1 * np.exp(-2 * np.pi * 1j * freqs)) ** 2


def _ar1_from_moments(c0: float, c1: float, N: int):
    """pycwt ar1 after the lag-0/lag-1 covariances."""
    B = -c1 * N - c0 * N ** 2 - 2 * c0 + 2 * c1 - c1 * N ** 2 + c0 * N
    A = c0 * N ** 2
    Cc = N * (c0 + c1 * N - c1)
    D = B ** 2 - 4 * A * Cc
    if D > 0:
        g = (-B - D ** 0.5) / (2 * A)
    else:
        raise Warning("Cannot place an upperbound on the unbiased AR(1). "
                      "Series is too short or trend is to large.")
    mu2 = -1 / N + (2 / N ** 2) * ((N - g ** N) / (1 - g) - g * (1 - g ** (N - 1)) / (1 - g) ** 2)
    c0t_pos = c0 / (1 - mu2)
    a = ((1 - g ** 2) * c0t_pos) ** 0.5
    return g, a, mu2


def ar1(x):
    """Unbiased AR(1) (g, a, mu2); covariances reduced on the GPU in fp64.
    Raises the built-in ``Warning`` like pycwt (the app's CPI fallback relies on it)."""
    xd = _to_dev(x)
    m = _np(ops.series_moments(xd.reshape(1, -1)))[0]
    return _ar1_from_moments(float(m[4]), float(m[5]), int(m[6]))


def significance(signal, dt, scales, sigma_test=0, alpha=None, significance_level=0.95,
                 dof=-1, wavelet="morlet"):
    """pycwt ``significance`` for sigma_test == 0 (the only form the reference uses)."""
    wavelet = as_mother(wavelet)
    try:
        n0 = len(signal)
    except TypeError:
        n0 = 1
    if n0 == 1:
        variance = signal
    else:
        m = _np(ops.series_moments(_to_dev(signal).reshape(1, -1)))[0]
        variance = m[1] ** 2
    if alpha is None:
        alpha, _, _ = ar1(signal)
    if sigma_test != 0:
        raise NotImplementedError("sigma_test != 0 is not used by the reference")
    period = np.asarray(scales) * wavelet.flambda()
    freq = dt / period
    fft_theor = variance * (1 - alpha ** 2) / (1 + alpha ** 2 - 2 * alpha * np.cos(2 * np.pi * freq))
    dof = wavelet.dofmin
    signif = fft_theor * _chi2_ppf(significance_level, dof) / dof
    return signif, fft_theor


# ------------------------------------------------------------- standardisation
def standardize_coefs(mom: torch.Tensor, detrend=True, standardize=True, remove_mean=False):
    """[B,3] affine coefficients reproducing ``standardize_series`` from [B,8] moments."""
    if detrend and remove_mean:
        raise ValueError("Only standardize by either removing secular trend or mean, not both.")
    B = mom.shape[0]
    coef = torch.zeros((B, 3), dtype=torch.float64, device=mom.device)
    if detrend:
        coef[:, 0] = mom[:, 3]
        coef[:, 1] = mom[:, 2]
    elif remove_mean:
        coef[:, 0] = mom[:, 0]
    coef[:, 2] = 1.0 / mom[:, 1] if standardize else 1.0
    return coef


def normalize_coefs(mom: torch.Tensor) -> torch.Tensor:
    """pycwt xwt/wct normalisation (y - mean) / std."""
    coef = torch.zeros((mom.shape[0], 3), dtype=torch.float64, device=mom.device)
    coef[:, 0] = mom[:, 0]
    coef[:, 2] = 1.0 / mom[:, 1]
    return coef


def standardize_series_dev(y: torch.Tensor, detrend=True, standardize=True, remove_mean=False,
                           dtype=torch.float64) -> torch.Tensor:
    y = y if y.dim() == 2 else y.reshape(1, -1)
    coef = ops.series_affine(y, (ops.AFF_DETREND if detrend else 0) | (ops.AFF_REMOVE_MEAN if remove_mean else 0)
                             | (ops.AFF_STANDARDIZE if standardize else 0))
    return ops.affine(y, coef, dtype)


def standardize_series(series, detrend=True, standardize=True, remove_mean=False):
    """GPU ``standardize_series`` (src/utils/wavelet_helpers.py:22-57), NumPy in/out."""
    if detrend and remove_mean:
        raise ValueError("Only standardize by either removing secular trend or mean, not both.")
    s = np.asarray(series)
    out = standardize_series_dev(_to_dev(s), detrend, standardize, remove_mean)
    return _np(out)[0]


# -------------------------------------------------------------------------- CWT
def cwt_batch(x: torch.Tensor, dt, dj=1 / 12, s0=-1, J=-1, wavelet="morlet", *, affine=None,
              sig_scale=None, want_w=True, want_power=False, want_sig=False):
    """Batched CWT of device rows (any pycwt mother: Morlet, Paul, DOG / MexicanHat);
    returns (dict of device tensors, sj, freqs)."""
    wavelet = as_mother(wavelet)
    n0 = x.shape[-1]
    sj, freqs = scales_for(n0, dt, dj, s0, J, wavelet)
    res = ops.cwt_morlet(x, sj, dt, affine=affine, sig_scale=sig_scale, want_w=want_w,
                         want_power=want_power, want_sig=want_sig, mother=wavelet)
    return res, sj, freqs


def cwt(signal, dt, dj=1 / 12, s0=-1, J=-1, wavelet="morlet", freqs=None):
    """pycwt-compatible ``cwt``: (W, sj, freqs, coi, signal_ft, ftfreqs), any pycwt mother."""
    wavelet = as_mother(wavelet)
    sig = np.asarray(signal)
    n0 = sig.size
    if freqs is not None:
        freqs = np.asarray(freqs, dtype=float)
        sj = 1 / (wavelet.flambda() * freqs)
    else:
        sj, freqs = scales_for(n0, dt, dj, s0, J, wavelet)
    xd = _to_dev(sig).reshape(1, -1)
    x32 = ops.affine(xd, torch.tensor([[0.0, 0.0, 1.0]], dtype=torch.float64, device=xd.device),
                     torch.float32)
    W = ops.cwt_morlet(x32, sj, dt, want_w=True, mother=wavelet)["w"][0]
    N = int(2 ** np.ceil(np.log2(n0)))
    ft = torch.fft.fft(xd[0], n=N)
    ftfreqs = 2 * np.pi * np.fft.fftfreq(N, dt)
    return (_np(W, np.complex128), sj, freqs, cone_of_influence(n0, dt, wavelet),
            _np(ft[1:N // 2]) / N ** 0.5, ftfreqs[1:N // 2] / (2 * np.pi))


# ----------------------------------------------------------------- XWT / WCT
def _pair_norm(y1, y2):
    d1, d2 = _to_dev(y1).reshape(1, -1), _to_dev(y2).reshape(1, -1)
    m1, m2 = ops.series_moments(d1), ops.series_moments(d2)
    return d1, d2, m1, m2


def xwt(y1, y2, dt, dj=1 / 12, s0=-1, J=-1, significance_level=0.95, wavelet="morlet",
        normalize=True):
    """pycwt-compatible ``xwt``: (W12, coi, freq, signif), any pycwt mother."""
    wavelet = as_mother(wavelet)
    d1, d2, m1, m2 = _pair_norm(y1, y2)
    n0 = d1.shape[1]
    sj, freq = scales_for(n0, dt, dj, s0, J, wavelet)
    if normalize:
        a1, a2 = normalize_coefs(m1), normalize_coefs(m2)
    else:
        ident = torch.tensor([[0.0, 0.0, 1.0]], dtype=torch.float64, device=d1.device)
        a1 = a2 = ident
    x1 = ops.affine(d1, a1, torch.float32)
    x2 = ops.affine(d2, a2, torch.float32)
    W12 = ops.xwt_morlet(x1, x2, sj, dt, want_w12=True, mother=wavelet)["w12"][0]
    mh1, mh2 = _np(m1)[0], _np(m2)[0]
    # pycwt resets std1 = std2 = 1 for normalised series (unit variance after the transform);
    # the raw deviations scale the test only when normalize=False
    std1, std2 = (1.0, 1.0) if normalize else (mh1[1], mh2[1])
    g1, _, _ = _ar1_from_moments(mh1[4], mh1[5], int(mh1[6]))
    g2, _, _ = _ar1_from_moments(mh2[4], mh2[5], int(mh2[6]))
    Pk1 = ar1_spectrum(freq * dt, g1)
    Pk2 = ar1_spectrum(freq * dt, g2)
    dof = wavelet.dofmin
    signif = std1 * std2 * (Pk1 * Pk2) ** 0.5 * _chi2_ppf(significance_level, dof) / dof
    return _np(W12, np.complex128), cone_of_influence(n0, dt, wavelet), freq, signif


def boxcar_rows(wavelet: Morlet, dj: float) -> int:
    """Morlet.smooth scale window length: int(round(2 * deltaj0 / dj))."""
    return int(np.round(wavelet.deltaj0 / dj * 2))


def wct_batch(y1: torch.Tensor, y2: torch.Tensor, dt, dj=1 / 12, s0=-1, J=-1, wavelet="morlet",
              normalize=True, want_uv=True, want_power=False, want_phase=False, workspace=None):
    """Batched coherence of device row pairs: (dict coh/u/v, sj, freqs)."""
    wavelet = as_morlet(wavelet)
    if wavelet.deltaj0 <= 0:
        raise ValueError("smoothing needs a Morlet(6) wavelet (deltaj0 defined)")
    n0 = y1.shape[-1]
    sj, freqs = scales_for(n0, dt, dj, s0, J, wavelet)
    a1 = a2 = None
    fused = normalize and 8 < n0 <= 16384  # normalised inside the transform's first kernel
    if normalize and not fused:
        a1 = ops.series_affine(y1, ops.AFF_NORMALIZE)
        a2 = ops.series_affine(y2, ops.AFF_NORMALIZE)
    res = ops.wct_morlet(y1, y2, sj, dt, wavelet.f0, boxcar=boxcar_rows(wavelet, dj), affine1=a1,
                         affine2=a2, want_uv=want_uv, want_power=want_power,
                         want_phase=want_phase, workspace=workspace, normalize=fused)
    return res, sj, freqs


def wct(y1, y2, dt, dj=1 / 12, s0=-1, J=-1, sig=True, significance_level=0.95,
        wavelet="morlet", normalize=True, **kwargs):
    """pycwt-compatible ``wct``: (WCT, aWCT, coi, freq, sig).  ``**kwargs`` reach
    ``wct_significance`` when ``sig`` (``cache=``, ``mc_count=``, ``seed=``) and are
    otherwise swallowed as in pycwt (``delta_j=`` -- reference quirk B.5)."""
    wavelet = as_morlet(wavelet)
    if np.asarray(y1).size != np.asarray(y2).size:
        raise AssertionError("Input signals must have the same size")
    d1, d2 = _to_dev(y1).reshape(1, -1), _to_dev(y2).reshape(1, -1)
    x1 = _norm32(d1) if normalize else d1.to(torch.float32)
    x2 = _norm32(d2) if normalize else d2.to(torch.float32)
    res, sj, freq = wct_batch(x1, x2, dt, dj, s0, J, wavelet, normalize=False, want_uv=False,
                              want_phase=True)
    n0 = d1.shape[1]
    if sig:
        if s0 == -1:
            s0 = 2 * dt / wavelet.flambda()
        if J == -1:
            J = int(np.round(np.log2(n0 * dt / s0) / dj))
        a1, _, _ = ar1(y1)
        a2, _, _ = ar1(y2)
        kw = {k: v for k, v in kwargs.items()
              if k in ("cache", "mc_count", "seed", "progress", "noise", "quantile")}
        sig = wct_significance(a1, a2, dt=dt, dj=dj, s0=s0, J=J,
                               significance_level=significance_level, wavelet=wavelet, **kw)
    else:
        sig = np.asarray([0])
    return (_np(res["coh"][0], np.float64), _np(res["phase"][0], np.float64),
            cone_of_influence(n0, dt, wavelet), freq, sig)


# ------------------------------------------------------ WCT Monte-Carlo significance
_GEOM_CACHE: dict = {}


def wct_sig_geometry(dt, dj, s0, J, wavelet="morlet"):
    """pycwt wct_significance set-up: noise length N = ceil(6 s0 2^(J dj) / dt), scales,
    and per scale the interval [t_lo, t_hi) of points outside the cone of influence
    (period_s <= coi_t; the COI is a triangle, so the set is an interval);
    maxscale = last scale with any such point (the counter runs over s < maxscale).
    The COI rises over the first half of the row, so each interval's ends come from one
    binary search on that half with the very comparison pycwt makes (period <= coi);
    results are kept per argument set (the app repeats its settings)."""
    wavelet = as_morlet(wavelet)
    key = (float(dt), float(dj), float(s0), int(J), wavelet.f0)
    hit = _GEOM_CACHE.get(key)
    if hit is not None:
        return hit[0], hit[1].copy(), hit[2].copy(), hit[3].copy(), hit[4].copy(), hit[5]
    ms = s0 * (2 ** (J * dj)) / dt
    N = int(np.ceil(ms * 6))
    sj = s0 * 2 ** (np.arange(0, J + 1) * dj)
    period = wavelet.flambda() * sj
    coi = cone_of_influence(N, dt, wavelet)
    half = (N + 1) // 2  # coi[:half] is non-decreasing, coi[t] == coi[N - 1 - t]
    rise = np.maximum.accumulate(coi[:half])
    first = np.searchsorted(rise, period, side="left")  # first t with coi[t] >= period
    # pycwt's own comparison decides the boundary samples (rounding of the triangle)
    for s in range(J + 1):
        t = int(first[s])
        while t > 0 and period[s] <= coi[t - 1]:
            t -= 1
        while t < half and not (period[s] <= coi[t]):
            t += 1
        first[s] = t
    anyout = first < half
    t_lo = np.where(anyout, first, 0).astype(np.int32)
    t_hi = np.where(anyout, N - first, 0).astype(np.int32)
    if not anyout.any():
        raise ValueError("no scale has points outside the cone of influence")
    maxscale = int(np.nonzero(anyout)[0][-1])
    if len(_GEOM_CACHE) >= 64:  # bounded: drop the oldest argument set (dicts keep order)
        _GEOM_CACHE.pop(next(iter(_GEOM_CACHE)), None)
    _GEOM_CACHE[key] = (N, sj, t_lo, t_hi, anyout, maxscale)
    return N, sj.copy(), t_lo.copy(), t_hi.copy(), anyout.copy(), maxscale


def significance_from_histogram(wlc: np.ndarray, anyout: np.ndarray, maxscale: int,
                                significance_level: float = 0.95) -> np.ndarray:
    """Per-scale coherence level at ``significance_level`` from the Monte-Carlo counters,
    as pycwt: NaN where a scale has points outside the COI, then for s < maxscale the
    quantile interpolated over the non-empty bins (P = (cumsum - 0.5) / total) on the
    mid-bin grid (b + 0.5) / nbins."""
    nbins = wlc.shape[1]
    sig95 = np.zeros(anyout.size)
    sig95[anyout] = np.nan
    if maxscale < 1:
        return sig95
    r2y = (np.arange(nbins) + 0.5) / nbins
    # all scales at once: np.interp over each scale's non-empty bins, i.e. the first
    # non-empty bin whose P reaches the level and the non-empty bin before it
    w = np.asarray(wlc[:maxscale], dtype=np.float64)
    nz = w != 0
    cum = np.cumsum(w, axis=1)
    tot = cum[:, -1:]
    with np.errstate(invalid="ignore", divide="ignore"):
        P = (cum - 0.5) / tot
    reach = nz & (P >= significance_level)
    hi = np.where(reach.any(axis=1), reach.argmax(axis=1), nbins - 1)
    idx = np.where(nz, np.arange(nbins), -1)
    prev = np.maximum.accumulate(idx, axis=1)  # last non-empty bin at or before each bin
    rows = np.arange(maxscale)
    has = reach.any(axis=1)
    lastnz = prev[:, -1]
    lo = np.where(hi > 0, prev[rows, np.maximum(hi - 1, 0)], -1)
    h = np.where(has, hi, np.maximum(lastnz, 0))
    lo_c = np.maximum(lo, 0)
    p0, p1 = P[rows, lo_c], P[rows, h]
    with np.errstate(invalid="ignore", divide="ignore"):
        lin = r2y[lo_c] + (significance_level - p0) * (r2y[h] - r2y[lo_c]) / (p1 - p0)
    # np.interp clamps outside the points: below the first non-empty bin -> its value, above
    # the last -> the last's; a scale with no counts keeps pycwt's initial value
    out = np.where(has & (lo >= 0), lin, r2y[h])
    out = np.where(lastnz < 0, sig95[:maxscale], out)
    sig95[:maxscale] = out
    return sig95


_sig_cache: dict = {}
_sig_cache_lock = threading.Lock()
# WTMI_WCT_SIG_CACHE=0 turns the significance cache off process-wide (latency
# measurements of the uncached Monte Carlo; callers' cache=True is then ignored)
SIG_CACHE = os.environ.get("WTMI_WCT_SIG_CACHE", "1") != "0"


def sig_cache_dir() -> str:
    """Directory of the persistent significance cache: $WTMI_CACHE_DIR, else
    ~/.cache/wtmi/wct_sig (pycwt keeps its own under the user cache dir)."""
    root = os.environ.get("WTMI_CACHE_DIR") or os.path.join(os.path.expanduser("~"), ".cache", "wtmi")
    return os.path.join(root, "wct_sig")


def _sig_cache_path(key) -> str:
    import hashlib
    h = hashlib.sha256(repr(key).encode()).hexdigest()[:32]
    return os.path.join(sig_cache_dir(), f"sig95_{h}.npy")


def sig_cache_load(key):
    """sig95 for a wct_significance argument key: process memory first, then disk."""
    with _sig_cache_lock:
        if key in _sig_cache:
            return _sig_cache[key].copy()
    path = _sig_cache_path(key)
    if os.path.exists(path):
        try:
            arr = np.load(path, allow_pickle=False)
        except (OSError, ValueError):
            return None  # unreadable entry: recompute (and overwrite it)
        with _sig_cache_lock:
            _sig_cache[key] = arr.copy()
        return arr
    return None


def sig_cache_store(key, sig95) -> None:
    """Keep sig95 in memory and on disk (atomic rename; a failed write only costs a
    recomputation later)."""
    import tempfile
    with _sig_cache_lock:
        _sig_cache[key] = np.array(sig95, copy=True)
    d = sig_cache_dir()
    try:
        os.makedirs(d, exist_ok=True)
        fd, tmp = tempfile.mkstemp(dir=d, suffix=".npy")
        with os.fdopen(fd, "wb") as fh:
            np.save(fh, np.asarray(sig95, dtype=np.float64), allow_pickle=False)
        os.replace(tmp, _sig_cache_path(key))
    except OSError:
        pass


# Monte-Carlo noise of wct_significance: "pycwt" (default) reproduces pycwt 0.4.0b0's
# helpers.rednoise as published -- lfilter along the length-1 axis of randn(N + tau, 1), i.e.
# white normals -- and "red" the AR(1) noise of Grinsted's MATLAB rednoise.m that it was ported
# from ("Monte-Carlo noise"; parity unpinned: pycwt is absent from the image).
SIG_NOISE = os.environ.get("WTMI_SIG_NOISE", "pycwt")

# Quantile step of wct_significance ("Monte-Carlo quantile"; parity unpinned):
# "pycwt" (default) is pycwt 0.4.0b0's published step: after the Monte-Carlo passes it masks
# the empty bins of its np.ma counter (``wlc.mask = (wlc.data == 0.)``) and, per scale,
# np.interp's the level over the non-empty bins (P = (cumsum - 0.5) / total on the mid-bin grid)
# -- ops.coherence_quantile on the device.  "nonempty" is the same rule under its r01-r05 name.
# "unmasked" is the explicit alternative reading without that mask line (the counter's mask is
# np.ma.nomask, ``~wlc[s, :].mask`` the scalar True, R2y[sel] 2-D): np.interp raises
# ValueError("object too deep for desired array") -- what r05 made the default.  The reference's
# own script (src/wct.py:453-465) and the app's significance checkbox (app/ui.py:74-81 ->
# src/wavelet_plots.py:510-514) plot levels from this call, so the masked reading is the default.
QUANTILE_MODES = ("pycwt", "nonempty", "unmasked")
SIG_QUANTILE = os.environ.get("WTMI_SIG_QUANTILE", "pycwt")
PYCWT_QUANTILE_ERROR = "object too deep for desired array"


def wct_significance(al1, al2, dt, dj, s0, J, significance_level=0.95, wavelet="morlet",
                     mc_count=300, progress=True, cache=True, seed=None, nbins=1000,
                     max_pairs_per_launch=512, noise=None, quantile=None):
    """pycwt ``wct_significance`` on the GPU: mc_count passes of two noise series
    (helpers.rednoise with al1, al2; ``noise`` "pycwt" or "red", default ``SIG_NOISE``),
    their coherence, and the per-scale counter of floor(R2 * nbins) outside the COI, batched
    max_pairs_per_launch passes per launch.  ``cache`` keeps results keyed on every argument,
    in process memory and on disk (``sig_cache_dir()``), as pycwt's ``cache=True`` keeps them
    under the user cache dir (src/wct.py:117); ``seed`` None draws a fresh one, as pycwt's
    unseeded draws do.  Like pycwt's rednoise (whose g == 0 branch calls the nonexistent
    ``np.randn``), a zero lag-1 coefficient raises AttributeError in the "pycwt" mode.
    ``quantile`` (``QUANTILE_MODES``, default ``SIG_QUANTILE`` = "pycwt"): "pycwt" and its
    alias "nonempty" interpolate each scale's level over its non-empty bins, as pycwt's masked
    counter selects them; "unmasked" raises ValueError once maxscale > 0, as pycwt's step would
    without its mask line (it would raise after the passes, which change nothing observable,
    so they are not run).  Cache order: pycwt reads its cache file before the Monte Carlo, and
    so does this call (a hit returns before any launch)."""
    wavelet = as_morlet(wavelet)
    if wavelet.deltaj0 <= 0:
        raise ValueError("wct_significance needs a Morlet(6) wavelet (deltaj0 defined)")
    noise = SIG_NOISE if noise is None else noise
    if noise not in ops.NOISE_MODES:
        raise ValueError(f"noise must be one of {ops.NOISE_MODES}, got {noise!r}")
    quantile = SIG_QUANTILE if quantile is None else quantile
    if quantile not in QUANTILE_MODES:
        raise ValueError(f"quantile must be one of {QUANTILE_MODES}, got {quantile!r}")
    if noise == "pycwt" and int(mc_count) > 0 and (float(al1) == 0.0 or float(al2) == 0.0):
        raise AttributeError("module 'numpy' has no attribute 'randn' "
                             "(pycwt helpers.rednoise with g == 0)")
    N, sj, t_lo, t_hi, anyout, maxscale = wct_sig_geometry(dt, dj, s0, J, wavelet)
    if quantile == "nonempty":
        quantile = "pycwt"  # one rule, one cache entry
    if quantile == "unmasked" and maxscale > 0:
        raise ValueError(f"{PYCWT_QUANTILE_ERROR} (quantile='unmasked': np.interp over the "
                         "np.ma counter without pycwt's wlc.mask = (wlc.data == 0.); the "
                         "default quantile='pycwt' gives the levels)")
    # the key holds the exact lag-1 coefficients (pycwt's cache name rounds arctanh(4 al),
    # NaN for |al| > 0.25)
    cache = cache and SIG_CACHE
    key = ("wct_significance", 3, noise, quantile, float(al1), float(al2), float(dt), float(dj),
           float(s0), int(J), float(significance_level), wavelet.f0, int(mc_count), int(nbins), seed)
    if cache:
        hit = sig_cache_load(key)
        if hit is not None:
            return hit
    if N > ops.MAX_SAMPLES:
        raise ValueError(f"wct_significance: noise length {N} exceeds the engine's "
                         f"{ops.MAX_SAMPLES} samples per row")
    # pairs per launch: all passes in one launch while the workspace (about 24 B per pair,
    # scale and sample) stays under 8 GiB -- the app's 300 passes of ~8k-sample noise take
    # one; long noise rows are split into several launches
    per_pair = max(1, ops.wct_workspace_bytes(1, N, sj.size))
    max_pairs_per_launch = int(max(1, min(max_pairs_per_launch, (8 << 30) // per_pair)))
    if seed is None:
        seed = int(np.random.SeedSequence().entropy) & ((1 << 64) - 1)
    dev = device()
    lo = torch.as_tensor(t_lo, device=dev)
    hi = torch.as_tensor(t_hi, device=dev)
    hist = torch.zeros((max(maxscale, 1), nbins), dtype=torch.int32, device=dev)
    K = boxcar_rows(wavelet, dj)
    ws = None
    for p0 in range(0, int(mc_count), max_pairs_per_launch):
        B = min(max_pairs_per_launch, int(mc_count) - p0)
        n1 = ops.rednoise(B, N, al1, seed, first_series=p0, device=dev, noise=noise)
        n2 = ops.rednoise(B, N, al2, seed, first_series=int(mc_count) + p0, device=dev, noise=noise)
        need = ops.wct_workspace_bytes(B, N, sj.size)
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=dev)
        coh = ops.wct_morlet(n1, n2, sj, dt, wavelet.f0, boxcar=K, want_uv=False, workspace=ws)["coh"]
        if maxscale > 0:
            ops.coherence_histogram(coh, lo, hi, maxscale, nbins, hist=hist)
    # the quantile step on the device (ops.coherence_quantile: the rule of
    # significance_from_histogram); only maxscale levels come back
    sig95 = np.zeros(sj.size)
    sig95[anyout] = np.nan
    if maxscale > 0:
        sig95[:maxscale] = _np(ops.coherence_quantile(hist, maxscale, significance_level))
    if cache:
        sig_cache_store(key, sig95)
    return sig95


def _norm32(d: torch.Tensor) -> torch.Tensor:
    """(y - mean) / std in fp64 on the device, rounded once to fp32."""
    return ops.affine(d, ops.series_affine(d, ops.AFF_NORMALIZE), torch.float32)


# ------------------------------------------------------------------------- DWT
def dwt_max_level(data_len: int, filter_len) -> int:
    if not isinstance(filter_len, (int, np.integer)):
        filter_len = as_filter_bank(filter_len).dec_len
    if filter_len < 2:
        raise ValueError("invalid wavelet filter length")
    if data_len < filter_len - 1:
        return 0
    return int(np.floor(np.log2(data_len / (filter_len - 1))))


def wavedec(data, wavelet, mode="symmetric", level=None):
    """pywt-compatible ``wavedec`` (mode 'symmetric' only): [cA_n, cD_n, ..., cD_1]."""
    if mode != "symmetric":
        raise ValueError("only mode='symmetric' (the reference's) is implemented")
    w = as_filter_bank(wavelet)
    x = np.asarray(data)
    if level is None:
        level = dwt_max_level(x.size, w.dec_len)
    if level < 0:
        raise ValueError(f"Level value of {level} is too low . Minimum level is 0.")
    xd = _to_dev(x, torch.float32).reshape(1, -1)
    coeffs, lens = ops.wavedec(xd, w.dec_lo, w.dec_hi, level)
    flat = _np(coeffs[0], np.float64)
    out, off = [], 0
    for L in lens:
        out.append(flat[off:off + L])
        off += L
    return out


def wavedec_batch(rows, wavelet, level=None):
    """wavedec of several series of one length in ONE launch: list of coefficient lists."""
    w = as_filter_bank(wavelet)
    x = np.asarray(rows)
    if x.ndim != 2:
        raise ValueError("wavedec_batch expects [batch, n]")
    if level is None:
        level = dwt_max_level(x.shape[1], w.dec_len)
    if level < 0:
        raise ValueError(f"Level value of {level} is too low . Minimum level is 0.")
    coeffs, lens = ops.wavedec(_to_dev(x, torch.float32), w.dec_lo, w.dec_hi, level)
    flat = _np(coeffs, np.float64)
    offs = np.concatenate([[0], np.cumsum(lens)])
    return [[flat[b, offs[k]:offs[k + 1]] for k in range(len(lens))] for b in range(x.shape[0])]


def _pack_coeffs(coeffs, dec_len):
    arrs = [np.asarray(c, dtype=np.float64) for c in coeffs]
    level = len(arrs) - 1
    # recover n from the finest detail length: len(cD_1) = (n + F - 1) // 2
    # (n is ambiguous by one; the synthesis only needs the list lengths, which the
    # kernel re-derives from n -- pick the n that reproduces every length)
    d1 = arrs[-1].size if level > 0 else arrs[0].size
    for n in ((2 * d1 - dec_len + 1, 2 * d1 - dec_len + 2) if level > 0 else (d1,)):
        if n < 1:
            continue
        if ops.dwt_lengths(n, dec_len, level) == [a.size for a in arrs]:
            return np.concatenate(arrs), n, level
    raise ValueError("coefficient shape mismatch")


def waverec_variants(coeffs, wavelet, keep_masks):
    """Batched waverec: one reconstruction per keep mask (bit k keeps coeffs[k])."""
    w = as_filter_bank(wavelet)
    flat, n, level = _pack_coeffs(coeffs, w.dec_len)
    dev = device()
    ct = torch.as_tensor(flat.astype(np.float32), device=dev).reshape(1, -1)
    out = ops.waverec(ct, n, w.rec_lo, w.rec_hi, level, keep_masks)
    return _np(out[0], np.float64)


def waverec(coeffs, wavelet, mode="symmetric"):
    if mode != "symmetric":
        raise ValueError("only mode='symmetric' (the reference's) is implemented")
    return waverec_variants(coeffs, wavelet, [(1 << len(coeffs)) - 1])[0]


# ----------------------------------------------------------------------- MODWT
def modwt(x, wavelet, level):
    w = as_filter_bank(wavelet)
    a = np.asarray(x)
    out = ops.modwt(_to_dev(a, torch.float32).reshape(1, -1), w.dec_lo, w.dec_hi, int(level))
    return _np(out[0], a.dtype if a.dtype in (np.float32, np.float64) else np.float64)


def imodwt(wc, wavelet, keep_mask=None):
    w = as_filter_bank(wavelet)
    a = np.asarray(wc)
    out = ops.imodwt(_to_dev(a, torch.float32).unsqueeze(0), w.dec_lo, w.dec_hi, keep_mask)
    return _np(out[0], a.dtype if a.dtype in (np.float32, np.float64) else np.float64)
