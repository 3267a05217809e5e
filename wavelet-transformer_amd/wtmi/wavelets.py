"""Mother wavelets that cross the drop-in boundary.

The reference passes live third-party objects into the transform functions:
``pycwt.Morlet(6)`` (``constants/results_configs.py:31,54``, ``src/cwt.py:44``) and
``pywt.Wavelet("db4")`` or the string ``"db4"`` (``constants/results_configs.py:28``,
``src/modwt.py:132``, ``src/dwt.py:28``).  Neither library is needed here: this module
provides equivalents and duck-types foreign objects (``.f0`` / ``.flambda()`` for a
Morlet; ``.dec_lo`` / ``.dec_hi`` / ``.rec_lo`` / ``.rec_hi`` / ``.name`` for a filter
bank).
"""

from __future__ import annotations

import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


class Morlet:
    """Morlet mother wavelet with the pycwt 0.4.0b0 constants."""

    name = "Morlet"

    def __init__(self, f0: float = 6.0):
        self.f0 = float(f0)
        self.dofmin = 2
        if self.f0 == 6:
            self.cdelta, self.gamma, self.deltaj0 = 0.776, 2.32, 0.60
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def psi_ft(self, f):
        return (np.pi ** -0.25) * np.exp(-0.5 * (np.asarray(f) - self.f0) ** 2)

    def flambda(self) -> float:
        return (4 * np.pi) / (self.f0 + np.sqrt(2 + self.f0 ** 2))

    def coi(self) -> float:
        return 1.0 / np.sqrt(2)

    def __repr__(self):
        return f"Morlet(f0={self.f0:g})"


class _Unsupported:
    """Descriptor of a pycwt mother wavelet the engine does not transform (only the Morlet
    Fourier filter is built into the CWT kernels).  Carries pycwt 0.4.0b0's constants so
    that the reference's ``MOTHER_DICT`` keys exist (src/xwt.py:29-34, src/wct.py:36-41);
    passing one to a transform raises ValueError, as for any non-Morlet wavelet."""

    name = "unsupported"

    def __repr__(self):
        return f"{type(self).__name__}(m={self.m})"


class Paul(_Unsupported):
    """pycwt ``Paul(m=4)``: flambda = 4 pi / (2m + 1), coi = sqrt(2)."""

    name = "Paul"

    def __init__(self, m: int = 4):
        self.m, self.dofmin = m, 2
        if m == 4:
            self.cdelta, self.gamma, self.deltaj0 = 1.132, 1.17, 1.5
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def flambda(self) -> float:
        return (4 * np.pi) / (2 * self.m + 1)

    def coi(self) -> float:
        return np.sqrt(2)


class DOG(_Unsupported):
    """pycwt ``DOG(m=2)`` (derivative of Gaussian): flambda = 2 pi / sqrt(m + 1/2)."""

    name = "DOG"

    def __init__(self, m: int = 2):
        self.m, self.dofmin = m, 1
        if m == 2:
            self.cdelta, self.gamma, self.deltaj0 = 3.541, 1.43, 1.4
        elif m == 6:
            self.cdelta, self.gamma, self.deltaj0 = 1.966, 1.37, 0.97
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def flambda(self) -> float:
        return (2 * np.pi / np.sqrt(self.m + 0.5))

    def coi(self) -> float:
        return 1 / np.sqrt(2)


class MexicanHat(DOG):
    """pycwt ``MexicanHat()`` = DOG(m=2)."""

    name = "Mexican Hat"

    def __init__(self):
        super().__init__(2)


def as_morlet(wavelet) -> Morlet:
    """Accept a wtmi/pycwt Morlet object, the string 'morlet', or None (Morlet(6))."""
    if wavelet is None:
        return Morlet(6)
    if isinstance(wavelet, Morlet):
        return wavelet
    if isinstance(wavelet, str):
        if wavelet.lower() == "morlet":
            return Morlet(6)
        raise ValueError(f"unsupported mother wavelet {wavelet!r}: only Morlet is implemented")
    if hasattr(wavelet, "f0") and type(wavelet).__name__.lower() == "morlet":
        m = Morlet(float(wavelet.f0))
        return m
    raise ValueError(f"unsupported mother wavelet {wavelet!r}: only Morlet is implemented")


_FILTERS = None


def _table():
    global _FILTERS
    if _FILTERS is None:
        with open(os.path.join(_HERE, "filters.json")) as f:
            _FILTERS = json.load(f)["dec_lo"]
    return _FILTERS


def wavelist():
    return sorted(_table())


class Wavelet:
    """Orthogonal filter bank with the pywt attribute names (dec_lo, dec_hi, rec_lo,
    rec_hi, dec_len, name).  Taps are PyWavelets' (filters.json)."""

    def __init__(self, name: str):
        key = "db1" if name == "haar" and "haar" not in _table() else name
        if key not in _table():
            raise ValueError(f"Unknown wavelet name {name!r}")
        lo = np.asarray(_table()[key], dtype=np.float64)
        k = np.arange(lo.size)
        self.name = name
        self.dec_lo = lo
        self.rec_lo = lo[::-1].copy()
        self.rec_hi = ((-1.0) ** k) * lo
        self.dec_hi = self.rec_hi[::-1].copy()
        self.dec_len = self.rec_len = lo.size

    @property
    def filter_bank(self):
        return self.dec_lo, self.dec_hi, self.rec_lo, self.rec_hi

    def __repr__(self):
        return f"Wavelet({self.name!r})"


def as_filter_bank(wavelet) -> Wavelet:
    """Accept a name ('db4'), a wtmi Wavelet, or any pywt-like object."""
    if isinstance(wavelet, Wavelet):
        return wavelet
    if isinstance(wavelet, str):
        return Wavelet(wavelet)
    if all(hasattr(wavelet, a) for a in ("dec_lo", "dec_hi", "rec_lo", "rec_hi")):
        w = Wavelet.__new__(Wavelet)
        w.name = getattr(wavelet, "name", "custom")
        w.dec_lo = np.asarray(wavelet.dec_lo, dtype=np.float64)
        w.dec_hi = np.asarray(wavelet.dec_hi, dtype=np.float64)
        w.rec_lo = np.asarray(wavelet.rec_lo, dtype=np.float64)
        w.rec_hi = np.asarray(wavelet.rec_hi, dtype=np.float64)
        w.dec_len = w.rec_len = w.dec_lo.size
        return w
    raise ValueError(f"cannot interpret {wavelet!r} as a wavelet filter bank")
