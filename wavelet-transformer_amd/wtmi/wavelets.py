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


class Paul:
    """pycwt ``Paul(m=4)``: conj(psi_hat(f)) = 2^m / sqrt(m (2m-1)!) f^m e^-f H(f) (real),
    flambda = 4 pi / (2m + 1), coi = sqrt(2), dofmin 2.  Transformed by the CWT / XWT kernels
    (mother id 1, include/wtmi.h); pycwt gives it no ``smooth``, so coherence raises."""

    name = "Paul"
    kernel_id = 1

    def __init__(self, m: int = 4):
        self.m, self.dofmin = m, 2
        if m == 4:
            self.cdelta, self.gamma, self.deltaj0 = 1.132, 1.17, 1.5
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def psi_ft(self, f):
        f = np.asarray(f, dtype=float)
        fp = np.where(f > 0, f, 0.0)
        norm = 2 ** self.m / np.sqrt(self.m * np.prod(np.arange(2, 2 * self.m, dtype=float)))
        return norm * fp ** self.m * np.exp(-fp) * (f > 0)

    def flambda(self) -> float:
        return (4 * np.pi) / (2 * self.m + 1)

    def coi(self) -> float:
        return np.sqrt(2)

    def __repr__(self):
        return f"Paul(m={self.m})"


class DOG:
    """pycwt ``DOG(m=2)`` (derivative of Gaussian): psi_hat(f) = -i^m / sqrt(Gamma(m + 1/2))
    f^m e^(-f^2/2), flambda = 2 pi / sqrt(m + 1/2), coi = 1/sqrt(2), dofmin 1.  Transformed by
    the CWT / XWT kernels (mother id 2); no ``smooth`` (pycwt), so coherence raises."""

    name = "DOG"
    kernel_id = 2

    def __init__(self, m: int = 2):
        self.m, self.dofmin = m, 1
        if m == 2:
            self.cdelta, self.gamma, self.deltaj0 = 3.541, 1.43, 1.4
        elif m == 6:
            self.cdelta, self.gamma, self.deltaj0 = 1.966, 1.37, 0.97
        else:
            self.cdelta = self.gamma = self.deltaj0 = -1

    def psi_ft(self, f):
        from math import gamma
        f = np.asarray(f, dtype=float)
        return -(1j ** self.m) / np.sqrt(gamma(self.m + 0.5)) * f ** self.m * np.exp(-0.5 * f ** 2)

    def flambda(self) -> float:
        return (2 * np.pi / np.sqrt(self.m + 0.5))

    def coi(self) -> float:
        return 1 / np.sqrt(2)

    def __repr__(self):
        return f"{type(self).__name__}(m={self.m})"


class MexicanHat(DOG):
    """pycwt ``MexicanHat()`` = DOG(m=2)."""

    name = "Mexican Hat"

    def __init__(self):
        super().__init__(2)


Morlet.kernel_id = 0


class NoSmoothError(AttributeError, ValueError):
    """A coherence (Morlet.smooth) was asked of a mother pycwt gives no ``smooth`` method:
    pycwt.wct raises AttributeError there; the ValueError base keeps the older contract."""


def as_morlet(wavelet) -> Morlet:
    """Accept a wtmi/pycwt Morlet object, the string 'morlet', or None (Morlet(6)).  The
    coherence paths need it: pycwt defines ``smooth`` for Morlet only."""
    if wavelet is None:
        return Morlet(6)
    if isinstance(wavelet, Morlet):
        return wavelet
    if isinstance(wavelet, str):
        if wavelet.lower() == "morlet":
            return Morlet(6)
    elif hasattr(wavelet, "f0") and type(wavelet).__name__.lower() == "morlet":
        return Morlet(float(wavelet.f0))
    if isinstance(wavelet, (str, Paul, DOG)) or type(wavelet).__name__ in ("Paul", "DOG", "MexicanHat"):
        raise NoSmoothError(f"{wavelet!r} has no attribute 'smooth': the wavelet coherence "
                            "needs Morlet (pycwt defines Morlet.smooth only)")
    raise ValueError(f"unsupported mother wavelet {wavelet!r}")


_MOTHER_NAMES = {"morlet": lambda: Morlet(6), "paul": lambda: Paul(4), "dog": lambda: DOG(2),
                 "mexicanhat": MexicanHat}


def as_mother(wavelet):
    """Any mother the CWT / XWT kernels transform: wtmi or pycwt Morlet / Paul / DOG /
    MexicanHat objects (duck-typed on the class name and ``f0`` / ``m``), their lower-case
    names, or None (Morlet(6))."""
    if wavelet is None:
        return Morlet(6)
    if isinstance(wavelet, (Morlet, Paul, DOG)):
        return wavelet
    if isinstance(wavelet, str):
        key = wavelet.lower().replace(" ", "").replace("_", "")
        if key in _MOTHER_NAMES:
            return _MOTHER_NAMES[key]()
        raise ValueError(f"unsupported mother wavelet {wavelet!r}")
    cls = type(wavelet).__name__
    if cls == "Morlet" and hasattr(wavelet, "f0"):
        return Morlet(float(wavelet.f0))
    if cls == "Paul" and hasattr(wavelet, "m"):
        return Paul(int(wavelet.m))
    if cls == "MexicanHat":
        return MexicanHat()
    if cls == "DOG" and hasattr(wavelet, "m"):
        return DOG(int(wavelet.m))
    raise ValueError(f"unsupported mother wavelet {wavelet!r}")


def kernel_mother(wavelet):
    """(mother id, parameter) of the C ABI's wtmi_cwt_mother / wtmi_xwt_mother."""
    w = as_mother(wavelet)
    return (0, float(w.f0)) if isinstance(w, Morlet) else (w.kernel_id, float(w.m))


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
