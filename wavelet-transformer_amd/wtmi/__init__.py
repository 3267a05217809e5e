"""wtmi -- MI355X-native wavelet-transform engine.

Layers:
  _lib        ctypes binding of libwtmi.so (C ABI, include/wtmi.h)
  ops         batched device-tensor API (torch tensors on the GPU, no CPU fallback)
  transforms  pycwt / PyWavelets-shaped functions (NumPy in / NumPy out) built on ops
  wavelets    Morlet and orthogonal filter banks (duck-types pycwt / pywt objects)
The reference-compatible modules (``src.cwt``, ``src.xwt``, ``src.wct``, ``src.dwt``,
``src.modwt``) live beside this package and call ``transforms``.
"""

from .wavelets import Morlet, Wavelet, as_filter_bank, as_morlet, wavelist  # noqa: F401

__all__ = ["Morlet", "Wavelet", "as_filter_bank", "as_morlet", "wavelist"]
