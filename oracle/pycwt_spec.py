"""fp64 CPU restatement of the pycwt 0.4.0b0 numerics the reference calls.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``wavelet-transformer_amd/``)
imports this module; only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker / the
timed CPU baseline.

Provenance and pinning
----------------------
pycwt==0.4.0b0 (pinned at reference ``requirements.txt:33``, ``uv.lock:874-886``) is
NOT present in this container and cannot be fetched (no network).  This file
restates its published algorithm (Torrence & Compo 1998; Grinsted et al. 2004;
pycwt ``wavelet.py`` / ``mothers.py`` / ``helpers.py``) as summarised in
SURVEY.md Appendix A, using the same scipy primitives pycwt uses when pyfftw is
absent (``scipy.fftpack.fft/ifft/fftfreq``, ``scipy.signal.convolve2d``,
``scipy.stats.chi2``).

**Parity for CWT / XWT / WCT / AR(1) / significance is UNPINNED**: the reference's
own tests assert lengths only (``tests/test_cwt.py:30,34``, ``tests/test_xwt.py:48,53``).
The restatement is pinned by the analytic known-answer tests of SURVEY.md A.6
(``tests/test_oracle_cwt.py``).

Reference call sites (what these functions stand in for):
  * ``cwt``          <- ``src/cwt.py:110``, inside ``xwt``/``wct``
  * ``ar1``          <- ``src/cwt.py:106``
  * ``significance`` <- ``src/cwt.py:123-131``
  * ``xwt``          <- ``src/xwt.py:93-101``
  * ``wct``          <- ``src/wct.py:106-118``, ``src/xwt.py:122-134``
  * ``wct_significance`` / ``rednoise`` <- inside ``wct(sig=True)``, ``src/wct.py:106-118``
"""

from __future__ import annotations

import numpy as np
from scipy import fftpack
from scipy.signal import convolve2d
from scipy.stats import chi2


class Morlet:
    """Morlet mother wavelet, pycwt ``mothers.Morlet``.

    Used by the reference as ``pycwt.Morlet(f0=6)`` (``src/cwt.py:44``,
    ``constants/results_configs.py:31,54``).
    """

    name = "Morlet"

    def __init__(self, f0: float = 6.0):
        self.f0 = float(f0)
        self.dofmin = 2
        if self.f0 == 6:
            self.cdelta = 0.776
            self.gamma = 2.32
            self.deltaj0 = 0.60
        else:
            self.cdelta = -1
            self.gamma = -1
            self.deltaj0 = -1

    def psi_ft(self, f):
        # No Heaviside step: negative frequencies contribute (A.1).
        return (np.pi ** -0.25) * np.exp(-0.5 * (f - self.f0) ** 2)

    def flambda(self):
        return (4 * np.pi) / (self.f0 + np.sqrt(2 + self.f0 ** 2))

    def coi(self):
        return 1.0 / np.sqrt(2)

    def smooth(self, W, dt, dj, scales):
        """Time Gaussian (via FFT) then scale boxcar, SURVEY A.4 ``Morlet.smooth``."""
        m, n = W.shape
        npad = next_pow2(n)
        k = 2 * np.pi * fftpack.fftfreq(npad)
        k2 = k ** 2
        snorm = scales / dt
        F = np.exp(-0.5 * (snorm[:, np.newaxis] ** 2) * k2)
        smooth = fftpack.ifft(F * fftpack.fft(W, axis=1, n=npad), axis=1, n=npad)
        T = smooth[:, :n]
        if np.isreal(W).all():
            T = T.real
        wsize = self.deltaj0 / dj * 2
        win = rect(int(np.round(wsize)), normalize=True)
        return convolve2d(T, win[:, np.newaxis], "same")


class Paul:
    """Paul mother wavelet of order m, pycwt ``mothers.Paul`` (Torrence & Compo 1998,
    Table 1).  psi_ft(f) = 2^m / sqrt(m (2m-1)!) f^m exp(-f) H(f); Fourier wavelength
    4 pi / (2m + 1); e-folding time sqrt(2) s (``coi`` = sqrt(2)); dofmin 2; no ``smooth``
    (pycwt defines it for Morlet only).  Reached through ``MOTHER_DICT["paul"]``
    (reference src/xwt.py:29-34, src/wct.py:36-41, constants/results_configs.py:53-58)."""

    name = "Paul"

    def __init__(self, m: int = 4):
        self.m = int(m)
        self.dofmin = 2
        if self.m == 4:
            self.cdelta, self.gamma, self.deltaj0 = 1.132, 1.17, 1.50
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def psi_ft(self, f):
        f = np.asarray(f, dtype=float)
        norm = 2 ** self.m / np.sqrt(self.m * np.prod(np.arange(2, 2 * self.m, dtype=float)))
        return norm * np.where(f > 0, f, 0.0) ** self.m * np.exp(-np.where(f > 0, f, 0.0)) * (f > 0)

    def flambda(self):
        return 4 * np.pi / (2 * self.m + 1)

    def coi(self):
        return np.sqrt(2)


class DOG:
    """Derivative-of-Gaussian mother wavelet of order m, pycwt ``mothers.DOG``
    (m = 2: the Mexican hat, pycwt ``MexicanHat``).  psi_ft(f) = -i^m / sqrt(Gamma(m + 1/2))
    f^m exp(-f^2 / 2); Fourier wavelength 2 pi / sqrt(m + 1/2); e-folding time sqrt(2) s
    (``coi`` = 1/sqrt(2)); dofmin 1; no ``smooth``."""

    name = "DOG"

    def __init__(self, m: int = 2):
        self.m = int(m)
        self.dofmin = 1
        if self.m == 2:
            self.cdelta, self.gamma, self.deltaj0 = 3.541, 1.43, 1.40
        elif self.m == 6:
            self.cdelta, self.gamma, self.deltaj0 = 1.966, 1.37, 0.97
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def psi_ft(self, f):
        from scipy.special import gamma
        f = np.asarray(f, dtype=float)
        return -(1j ** self.m) / np.sqrt(gamma(self.m + 0.5)) * f ** self.m * np.exp(-0.5 * f ** 2)

    def flambda(self):
        return 2 * np.pi / np.sqrt(self.m + 0.5)

    def coi(self):
        return 1 / np.sqrt(2)


class MexicanHat(DOG):
    """pycwt ``mothers.MexicanHat``: DOG of order 2."""

    name = "Mexican Hat"

    def __init__(self):
        super().__init__(2)


def rect(x: int, normalize: bool = False) -> np.ndarray:
    """Boxcar with half-weight end points (pycwt ``helpers.rect``)."""
    X = np.zeros(x)
    X[0] = X[-1] = 0.5
    X[1:-1] = 1
    if normalize:
        X /= X.sum()
    return X


def next_pow2(n: int) -> int:
    """pycwt ``helpers.fft_kwargs``: FFT length = 2**ceil(log2(n))."""
    return int(2 ** np.ceil(np.log2(n)))


def scales_for(n0: int, dt: float, dj: float, s0: float, J: float, wavelet: Morlet):
    """Default-parameter resolution of pycwt ``cwt``."""
    if s0 == -1:
        s0 = 2 * dt / wavelet.flambda()
    if J == -1:
        J = int(np.round(np.log2(n0 * dt / s0) / dj))
    sj = s0 * 2 ** (np.arange(0, J + 1) * dj)
    freqs = 1 / (wavelet.flambda() * sj)
    return sj, freqs


def cwt(signal, dt, dj=1 / 12, s0=-1, J=-1, wavelet=None):
    """pycwt ``cwt``: FFT convolution with the analytic Morlet.

    Returns ``(W[:, :n0], sj, freqs, coi, signal_ft[1:N//2]/sqrt(N), ftfreqs[1:N//2]/2pi)``.
    """
    wavelet = wavelet or Morlet(6)
    signal = np.asarray(signal)
    n0 = len(signal)
    sj, freqs = scales_for(n0, dt, dj, s0, J, wavelet)
    N = next_pow2(n0)
    signal_ft = fftpack.fft(signal, n=N)
    ftfreqs = 2 * np.pi * fftpack.fftfreq(N, dt)
    sj_col = sj[:, np.newaxis]
    psi_ft_bar = (sj_col * ftfreqs[1] * N) ** 0.5 * np.conjugate(
        wavelet.psi_ft(sj_col * ftfreqs)
    )
    W = fftpack.ifft(signal_ft * psi_ft_bar, axis=1, n=N)
    sel = np.invert(np.isnan(W).all(axis=1))
    if np.any(sel):
        sj = sj[sel]
        freqs = freqs[sel]
        W = W[sel, :]
    coi = n0 / 2 - np.abs(np.arange(0, n0) - (n0 - 1) / 2)
    coi = wavelet.flambda() * wavelet.coi() * dt * coi
    return (
        W[:, :n0],
        sj,
        freqs,
        coi,
        signal_ft[1 : N // 2] / N ** 0.5,
        ftfreqs[1 : N // 2] / (2 * np.pi),
    )


def ar1(x):
    """Unbiased AR(1) estimate after Grinsted.

    Raises the built-in ``Warning`` when no upper bound exists; the reference
    app relies on catching it (``src/wavelet_plots.py:684``).
    """
    x = np.asarray(x)
    N = x.size
    xm = x.mean()
    x = x - xm
    c0 = x.transpose().dot(x) / len(x)
    c1 = x[0 : N - 1].transpose().dot(x[1:N]) / (N - 1)
    B = -c1 * N - c0 * N ** 2 - 2 * c0 + 2 * c1 - c1 * N ** 2 + c0 * N
    A = c0 * N ** 2
    C = N * (c0 + c1 * N - c1)
    D = B ** 2 - 4 * A * C
    if D > 0:
        g = (-B - D ** 0.5) / (2 * A)
    else:
        raise Warning(
            "Cannot place an upperbound on the unbiased AR(1). "
            "Series is too short or trend is to large."
        )
    mu2 = -1 / N + (2 / N ** 2) * (
        (N - g ** N) / (1 - g) - g * (1 - g ** (N - 1)) / (1 - g) ** 2
    )
    c0t_pos = c0 / (1 - mu2)
    a = ((1 - g ** 2) * c0t_pos) ** 0.5
    return g, a, mu2


def ar1_spectrum(freqs, ar1=0.0):
    freqs = np.asarray(freqs)
    return (1 - ar1 ** 2) / np.abs(1 - ar1 * np.exp(-2 * np.pi * 1j * freqs)) ** 2


def significance(signal, dt, scales, sigma_test=0, alpha=None,
                 significance_level=0.95, dof=-1, wavelet=None):
    """pycwt ``significance`` for ``sigma_test == 0`` (the only form the reference uses,
    ``src/cwt.py:123-131``)."""
    wavelet = wavelet or Morlet(6)
    try:
        n0 = len(signal)
    except TypeError:
        n0 = 1
    if n0 == 1:
        variance = signal
    else:
        variance = np.asarray(signal).std() ** 2
    if alpha is None:
        alpha, _, _ = ar1(signal)
    period = scales * wavelet.flambda()
    freq = dt / period
    dofmin = wavelet.dofmin
    fft_theor = (1 - alpha ** 2) / (1 + alpha ** 2 - 2 * alpha * np.cos(2 * np.pi * freq))
    fft_theor = variance * fft_theor
    if sigma_test != 0:
        raise NotImplementedError("only sigma_test=0 is used by the reference")
    dof = dofmin
    chisquare = chi2.ppf(significance_level, dof) / dof
    signif = fft_theor * chisquare
    return signif, fft_theor


def _normalized(y1, y2, normalize):
    y1 = np.asarray(y1)
    y2 = np.asarray(y2)
    std1 = y1.std()
    std2 = y2.std()
    if normalize:
        return y1, y2, (y1 - y1.mean()) / std1, (y2 - y2.mean()) / std2, std1, std2
    return y1, y2, y1, y2, std1, std2


def xwt(y1, y2, dt, dj=1 / 12, s0=-1, J=-1, significance_level=0.95,
        wavelet=None, normalize=True):
    """pycwt ``xwt``. Returns ``(W12, coi, freq, signif)``."""
    wavelet = wavelet or Morlet(6)
    y1, y2, y1n, y2n, std1, std2 = _normalized(y1, y2, normalize)
    kw = dict(dj=dj, s0=s0, J=J, wavelet=wavelet)
    W1, sj, freq, coi, _, _ = cwt(y1n, dt, **kw)
    W2, sj, freq, coi, _, _ = cwt(y2n, dt, **kw)
    W12 = W1 * W2.conj()
    # pycwt resets std1 = std2 = 1 when the series were normalised: the transformed series
    # then have unit variance, so their red-noise spectra are scaled by 1, not by the raw
    # variances (SURVEY A.4 step 4 omits this condition)
    if normalize:
        std1 = std2 = 1.0
    a1, _, _ = ar1(y1)
    a2, _, _ = ar1(y2)
    Pk1 = ar1_spectrum(freq * dt, a1)
    Pk2 = ar1_spectrum(freq * dt, a2)
    dof = wavelet.dofmin
    PPF = chi2.ppf(significance_level, dof)
    signif = std1 * std2 * (Pk1 * Pk2) ** 0.5 * PPF / dof
    return W12, coi, freq, signif


def wct(y1, y2, dt, dj=1 / 12, s0=-1, J=-1, sig=True, significance_level=0.95,
        wavelet=None, normalize=True, **kwargs):
    """pycwt ``wct``.

    ``**kwargs`` swallows ``cache=`` and ``delta_j=`` exactly as pycwt does
    (reference quirk B.5: ``src/xwt.py:126`` passes ``delta_j=`` and so runs at
    the default dj=1/12); ``mc_count`` / ``rng`` reach ``wct_significance``.
    """
    wavelet = wavelet or Morlet(6)
    if np.asarray(y1).size != np.asarray(y2).size:
        raise AssertionError("Input signals must have the same size")
    y1, y2, y1n, y2n, _, _ = _normalized(y1, y2, normalize)
    kw = dict(dj=dj, s0=s0, J=J, wavelet=wavelet)
    W1, sj, freq, coi, _, _ = cwt(y1n, dt, **kw)
    W2, sj, freq, coi, _, _ = cwt(y2n, dt, **kw)
    scales = np.ones([1, y1.size]) * sj[:, None]
    S1 = wavelet.smooth(np.abs(W1) ** 2 / scales, dt, dj, sj)
    S2 = wavelet.smooth(np.abs(W2) ** 2 / scales, dt, dj, sj)
    W12 = W1 * W2.conj()
    S12 = wavelet.smooth(W12 / scales, dt, dj, sj)
    WCT = np.abs(S12) ** 2 / (S1 * S2)
    aWCT = np.angle(W12)
    if sig:
        a1, _, _ = ar1(y1)
        a2, _, _ = ar1(y2)
        sig = wct_significance(a1, a2, dt=dt, dj=dj, s0=s0, J=J,
                               significance_level=significance_level, wavelet=wavelet,
                               **{k: v for k, v in kwargs.items() if k in ("mc_count", "rng", "noise", "quantile")})
    else:
        sig = np.asarray([0])
    return WCT, aWCT, coi, freq, sig


# ------------------------------------------------------------ Monte-Carlo significance
# pycwt 0.4.0b0 ``helpers.rednoise`` and ``wavelet.wct_significance`` (SURVEY A.5;
# reached from src/wct.py:106-118 with sig=True).  The published algorithm draws from
# the unseeded global ``np.random``; here the generator is a parameter so tests can
# seed it.  Parity with the GPU path is statistical (different random streams).

def rednoise(N: int, g: float, a: float = 1.0, rng=None, noise: str = "pycwt") -> np.ndarray:
    """pycwt 0.4.0b0 ``helpers.rednoise(N, g, a)``, restated from its published source:

        if g == 0: yr = np.randn(N, 1) * a          # AttributeError: numpy has no randn
        else:
            tau = int(np.ceil(-2 / np.log(np.abs(g))))
            yr = lfilter([1, 0], [1, -g], np.random.randn(N + tau, 1) * a)
            yr = yr[tau:]
        return yr.flatten()

    noise="pycwt" (default) does exactly that: scipy's lfilter filters along axis=-1, which has
    length 1 for the (N + tau, 1) array, so the call is the identity and the noise is WHITE
    (g only sets how many leading draws tau are dropped).  noise="red" filters along axis 0,
    the AR(1) red noise of Grinsted's MATLAB rednoise.m (MATLAB's filter works along the first
    non-singleton dimension), which the port meant.  DESIGN 4 records the choice; parity
    unpinned (pycwt is absent from the image)."""
    from scipy.signal import lfilter
    if noise not in ("pycwt", "red"):
        raise ValueError(noise)
    rng = rng if rng is not None else np.random.default_rng()
    if g == 0:
        if noise == "pycwt":
            raise AttributeError("module 'numpy' has no attribute 'randn'")
        return (rng.standard_normal((N, 1)) * a).flatten()
    tau = int(np.ceil(-2 / np.log(np.abs(g))))
    e = rng.standard_normal((N + tau, 1)) * a
    yr = lfilter([1, 0], [1, -g], e) if noise == "pycwt" else lfilter([1, 0], [1, -g], e, axis=0)
    return yr[tau:].flatten()


def wct_sig_geometry(dt, dj, s0, J, wavelet=None):
    """Noise length N = ceil(6 s0 2^(J dj) / dt), the outside-COI mask [J+1, N] and
    maxscale (last scale with any point outside the COI), as in wct_significance."""
    wavelet = wavelet or Morlet(6)
    ms = s0 * (2 ** (J * dj)) / dt
    N = int(np.ceil(ms * 6))
    sj = s0 * 2 ** (np.arange(0, J + 1) * dj)
    freq = 1 / (wavelet.flambda() * sj)
    coi = N / 2 - np.abs(np.arange(0, N) - (N - 1) / 2)
    coi = wavelet.flambda() * wavelet.coi() * dt * coi
    period = np.ones([1, N]) / freq[:, None]
    outsidecoi = period <= (np.ones([J + 1, 1]) * coi[None, :])
    maxscale = int(np.nonzero(outsidecoi.any(axis=1))[0][-1])
    return N, sj, outsidecoi, maxscale


def coherence_histogram(R2, outsidecoi, maxscale, nbins=1000, wlc=None):
    """One Monte-Carlo pass of the counter: for s < maxscale, bins floor(R2 * nbins)
    of the points outside the COI.  (pycwt indexes with int(floor(..)); R2 == 1.0
    exactly would raise IndexError there -- clamped to the last bin here.)"""
    J1 = R2.shape[0]
    wlc = np.zeros((J1, nbins)) if wlc is None else wlc
    for s in range(maxscale):
        cd = np.floor(R2[s, outsidecoi[s]] * nbins).astype(np.int64)
        np.add.at(wlc[s], np.clip(cd, 0, nbins - 1), 1)
    return wlc


PYCWT_QUANTILE_ERROR = "object too deep for desired array"


def significance_from_histogram(wlc, outsidecoi, maxscale, significance_level=0.95,
                                quantile="pycwt"):
    """sig95 from the per-scale counters: NaN for scales with points outside the COI, then
    the quantile step for s < maxscale.

    quantile="pycwt" (default) executes pycwt 0.4.0b0's published statements (DESIGN 4,
    "Monte-Carlo quantile"):

        wlc = np.ma.zeros([J + 1, nbins])
        ...                                        # wlc[s, int(t)] += 1 per outside-COI point
        wlc.mask = (wlc.data == 0.)                # after the Monte-Carlo loop: mask empty bins
        R2y = (np.arange(nbins) + 0.5) / nbins
        for s in range(maxscale):
            sel = ~wlc[s, :].mask                  # the scale's non-empty bins
            P = wlc[s, sel].data.cumsum()
            P = (P - 0.5) / P[-1]
            sig95[s] = np.interp(significance_level, P, R2y[sel])

    (the mask line is the Python form of Grinsted's wtcsignif.m ``idx=find(ptile~=0)``).
    quantile="nonempty" is the same rule written on a plain array.  quantile="unmasked" runs
    the statements without the mask line: the mask is then np.ma.nomask, ``sel`` the scalar
    True, R2y[sel] has shape (1, nbins) and np.interp raises ValueError("object too deep for
    desired array") -- r05's reading, kept as an explicit alternative.  Parity unpinned: pycwt
    is absent from the image (tests/test_wct_sig_host.py runs the lines under numpy 1.26.4)."""
    if quantile not in ("pycwt", "nonempty", "unmasked"):
        raise ValueError(quantile)
    nbins = wlc.shape[1]
    sig95 = np.zeros(wlc.shape[0])
    sig95[outsidecoi.any(axis=1)] = np.nan
    R2y = (np.arange(nbins) + 0.5) / nbins
    if quantile in ("pycwt", "unmasked"):
        counter = np.ma.zeros(wlc.shape)
        counter[:, :] = wlc
        if quantile == "pycwt":
            counter.mask = (counter.data == 0.)
        with np.errstate(invalid="ignore", divide="ignore"):
            for s in range(maxscale):
                sel = ~counter[s, :].mask
                P = counter[s, sel].data.cumsum()
                P = (P - 0.5) / P[-1]
                sig95[s] = np.interp(significance_level, P, R2y[sel])
        return sig95
    for s in range(maxscale):
        sel = wlc[s, :] != 0
        P = wlc[s, sel].cumsum()
        P = (P - 0.5) / P[-1]
        sig95[s] = np.interp(significance_level, P, R2y[sel])
    return sig95


def pycwt_cache_name(al1, al2, dt, dj, s0, J, wavelet_name="morlet"):
    """pycwt 0.4.0b0 ``wct_significance``'s cache file name, as published:

        aa = np.round(np.arctanh(np.array([al1, al2]) * 4))
        aa = np.abs(aa) + 0.5 * (aa < 0)
        cache = 'wct_sig_{:0.5f}_{:0.5f}_{:0.5f}_{:0.5f}_{:d}_{}'.format(
            aa[0], aa[1], dj, s0 / dt, J, wavelet.name)

    arctanh(4 al) is NaN for |al| > 0.25, so every such series shares the name's 'nan'
    fields (the engine keys on the exact al instead)."""
    with np.errstate(invalid="ignore", divide="ignore"):
        aa = np.round(np.arctanh(np.array([al1, al2]) * 4))
    aa = np.abs(aa) + 0.5 * (aa < 0)
    return "wct_sig_{:0.5f}_{:0.5f}_{:0.5f}_{:0.5f}_{:d}_{}".format(
        aa[0], aa[1], dj, s0 / dt, J, wavelet_name)


def wct_significance(al1, al2, dt, dj, s0, J, significance_level=0.95, wavelet=None,
                     mc_count=300, rng=None, nbins=1000, noise="pycwt", quantile="pycwt"):
    """pycwt ``wct_significance`` without the disk cache; ``noise`` as in
    ``rednoise``, ``quantile`` as in ``significance_from_histogram`` (the "unmasked" reading
    raises ValueError after the Monte Carlo whenever maxscale > 0)."""
    wavelet = wavelet or Morlet(6)
    rng = rng if rng is not None else np.random.default_rng()
    N, sj, outsidecoi, maxscale = wct_sig_geometry(dt, dj, s0, J, wavelet)
    scales = np.ones([1, N]) * sj[:, None]
    wlc = np.zeros((J + 1, nbins))
    kw = dict(dj=dj, s0=s0, J=J, wavelet=wavelet)
    for _ in range(mc_count):
        noise1 = rednoise(N, al1, 1, rng, noise)
        noise2 = rednoise(N, al2, 1, rng, noise)
        nW1, sj, _, _, _, _ = cwt(noise1, dt, **kw)
        nW2, sj, _, _, _, _ = cwt(noise2, dt, **kw)
        nW12 = nW1 * nW2.conj()
        S1 = wavelet.smooth(np.abs(nW1) ** 2 / scales, dt, dj, sj)
        S2 = wavelet.smooth(np.abs(nW2) ** 2 / scales, dt, dj, sj)
        S12 = wavelet.smooth(nW12 / scales, dt, dj, sj)
        R2 = np.abs(S12) ** 2 / (S1 * S2)
        coherence_histogram(R2, outsidecoi, maxscale, nbins, wlc)
    return significance_from_histogram(wlc, outsidecoi, maxscale, significance_level, quantile)
