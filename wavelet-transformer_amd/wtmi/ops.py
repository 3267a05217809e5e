"""Batched device-tensor API over libwtmi.so.

Every function takes/returns torch tensors resident on an MI355X (``cuda`` device
under ROCm), enqueues the HIP kernels on the current stream of that device and
returns without synchronising.  There is no CPU implementation: a CPU tensor or a
missing library raises.  The same functions are registered as torch custom ops
(``torch.ops.wtmi.*``, see ``_register``) so they compose with torch code.
"""

from __future__ import annotations

import ctypes as C
import threading
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib

VP = C.c_void_p


def _ptr(t: Optional[torch.Tensor]):
    return VP(t.data_ptr()) if t is not None else VP(None)


def _stream(dev: torch.device):
    return VP(torch.cuda.current_stream(dev).cuda_stream)


def _check_dev(*ts):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError(
                f"wtmi kernels run on the GPU only; got a tensor on {t.device} "
                "(no CPU fallback exists)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError("all wtmi operands must be on the same device")
    return dev


def _rows(x: torch.Tensor, dtype=None) -> torch.Tensor:
    """[n] or [B, n] -> [B, n] with unit stride along time and a row stride >= n (the C ABI's
    ld).  A size-1 batch dimension may carry any stride in torch (NumPy's x[None, :] arrives
    with stride 0), so a one-row view is re-strided to ld = n; an expanded batch is copied."""
    if dtype is not None:
        x = x.to(dtype)
    if x.dim() == 1:
        x = x.unsqueeze(0)
    if x.dim() != 2:
        raise ValueError("expected a [batch, n] tensor")
    B, n = x.shape
    if x.stride(1) != 1 or (B > 1 and x.stride(0) < n):
        x = x.contiguous()
    if B == 1 and x.stride(0) != n:
        x = x.as_strided((1, n), (n, 1), x.storage_offset())
    return x


_F64_CACHE: "dict[tuple, torch.Tensor]" = {}
_F64_CACHE_MAX = 256
_F64_LOCK = threading.Lock()


def _f64_dev(a, dev) -> Optional[torch.Tensor]:
    """Host arrays (scale vectors, significance multipliers) as device float64 tensors.
    A pageable host-to-device copy blocks the host until the stream drains, which
    serialises back-to-back transforms; the copies are therefore content-addressed and
    cached per device (the key is the array's bytes, so a changed array is a new entry)."""
    if a is None:
        return None
    if isinstance(a, torch.Tensor):
        return a.to(device=dev, dtype=torch.float64).contiguous()
    h = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    key = (str(dev), h.shape, h.tobytes())
    with _F64_LOCK:
        t = _F64_CACHE.get(key)
    if t is None:
        t = torch.as_tensor(h, device=dev)
        with _F64_LOCK:
            if len(_F64_CACHE) >= _F64_CACHE_MAX:
                _F64_CACHE.pop(next(iter(_F64_CACHE)))
            _F64_CACHE[key] = t
    # the cached block may be read by kernels on several streams: tell the caching
    # allocator about this one, so an eviction cannot recycle it under a running kernel
    t.record_stream(torch.cuda.current_stream(dev))
    return t


# ------------------------------------------------------------------------ moments
def series_moments(x: torch.Tensor) -> torch.Tensor:
    """[B, 8] float64: mean, std(ddof 0), slope, intercept, c0, c1, n, 0."""
    x = _rows(x)
    dev = _check_dev(x)
    if x.dtype not in (torch.float32, torch.float64):
        x = _rows(x, torch.float64)
    out = torch.empty((x.shape[0], 8), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_series_moments", _ptr(x), int(x.dtype == torch.float64), x.stride(0),
                  x.shape[0], x.shape[1], _ptr(out), _stream(dev))
    return out


AFF_DETREND, AFF_REMOVE_MEAN, AFF_STANDARDIZE = 1, 2, 4
AFF_NORMALIZE = AFF_REMOVE_MEAN | AFF_STANDARDIZE  # pycwt xwt / wct: (y - mean) / std


def series_affine(x: torch.Tensor, mode: int = AFF_NORMALIZE) -> torch.Tensor:
    """[B, 3] float64 affine coefficients (x - a0 - a1 t) * a2 from one moments pass (mode bits:
    1 detrend, 2 remove mean, 4 standardize; 1 and 2 together raise ValueError)."""
    if (mode & AFF_DETREND) and (mode & AFF_REMOVE_MEAN):
        raise ValueError("Only standardize by either removing secular trend or mean, not both.")
    x = _rows(x)
    dev = _check_dev(x)
    if x.dtype not in (torch.float32, torch.float64):
        x = _rows(x, torch.float64)
    out = torch.empty((x.shape[0], 3), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_series_affine", _ptr(x), int(x.dtype == torch.float64), x.stride(0),
                  x.shape[0], x.shape[1], int(mode), None, _ptr(out), _stream(dev))
    return out


def affine(x: torch.Tensor, coef: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """y = (x - a0 - a1 t) * a2 per series (coef [B, 3] float64), computed in fp64."""
    x = _rows(x)
    dev = _check_dev(x, coef)
    if x.dtype not in (torch.float32, torch.float64):
        x = _rows(x, torch.float64)
    coef = coef.to(torch.float64).contiguous()
    y = torch.empty(x.shape, dtype=dtype, device=dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_affine", _ptr(x), int(x.dtype == torch.float64), x.stride(0), x.shape[0],
                  x.shape[1], _ptr(coef), _ptr(y), int(dtype == torch.float64), y.stride(0),
                  _stream(dev))
    return y


# ---------------------------------------------------------------------------- CWT
# Operand checks run BEFORE anything touches a device: a wrong-sized buffer must never
# reach a kernel that indexes it by batch and scale (the kernels trust their geometry).
def _shape(a):
    return tuple(a.shape) if isinstance(a, torch.Tensor) else np.shape(a)


def _n_scales(scales) -> int:
    shp = _shape(scales)
    if scales is None or len(shp) != 1 or shp[0] < 1:
        raise ValueError(f"scales must be a non-empty 1-D array, got shape {shp}")
    return shp[0]


def _check_affine(a, B, name):
    if a is not None and (not isinstance(a, torch.Tensor) or tuple(a.shape) != (B, 3)):
        raise ValueError(f"{name} must be a [{B}, 3] tensor, got "
                         f"{tuple(a.shape) if isinstance(a, torch.Tensor) else type(a).__name__}")


def _check_sig(sig_scale, B, S, want_sig):
    """sig_scale: [S] (every series) or [B, S] (per series); returns sig_ld."""
    if not want_sig:
        return 0
    if sig_scale is None:
        raise ValueError("want_sig needs sig_scale")
    shp = _shape(sig_scale)
    if shp == (S,):
        return 0
    if shp == (B, S):
        return S
    raise ValueError(f"sig_scale must have shape [{S}] or [{B}, {S}], got {shp}")


def _check_out(out, shape, dtype, name):
    if out is not None and (not isinstance(out, torch.Tensor) or tuple(out.shape) != tuple(shape)
                            or out.dtype != dtype or not out.is_contiguous()):
        raise ValueError(f"{name} must be a contiguous {dtype} tensor of shape {tuple(shape)}, got "
                         f"{_shape(out)} {getattr(out, 'dtype', type(out).__name__)}")


def _f64_arg(a, dev):
    return None if a is None else a.to(device=dev, dtype=torch.float64).contiguous()


def _mother_args(mother, f0):
    """(id, parameter) for wtmi_cwt_mother / wtmi_xwt_mother: None -> Morlet(f0); else a
    wtmi / pycwt mother object or an (id, parameter) pair (wavelets.kernel_mother)."""
    if mother is None:
        return 0, float(f0)
    if isinstance(mother, tuple):
        return int(mother[0]), float(mother[1])
    from .wavelets import kernel_mother
    return kernel_mother(mother)


def cwt_morlet(x: torch.Tensor, scales, dt: float, f0: float = 6.0, *,
               affine: Optional[torch.Tensor] = None, sig_scale=None,
               want_w: bool = True, want_power: bool = False, want_sig: bool = False,
               out_w: Optional[torch.Tensor] = None, mother=None):
    """CWT of every row of x (float32 [B, n0]) at the given scales: Morlet(f0), or the
    pycwt mother ``mother`` (Paul / DOG / MexicanHat objects, wavelets.kernel_mother).

    Returns a dict with any of ``w`` (complex64 [B, S, n0]), ``power`` and ``sig``
    (float32 [B, S, n0], sig = power * sig_scale[j], or sig_scale[b, j] for a [B, S]
    sig_scale).  Every caller-supplied operand is checked against the launch geometry
    (shape, dtype, device, contiguity) before the kernel sees it.
    """
    x = _rows(x)
    B, n0 = x.shape
    S = _n_scales(scales)
    sig_ld = _check_sig(sig_scale, B, S, want_sig)
    _check_affine(affine, B, "affine")
    _check_out(out_w, (B, S, n0), torch.complex64, "out_w")
    if out_w is not None and not want_w:
        raise ValueError("out_w given with want_w=False")
    if not (want_w or want_power or want_sig):
        raise ValueError("cwt_morlet: no output requested")
    dev = _check_dev(x, affine, out_w)
    x = _rows(x, torch.float32)
    sc = _f64_dev(scales, dev)
    ss = _f64_dev(sig_scale, dev) if want_sig else None
    aff = _f64_arg(affine, dev)
    res = {}
    if want_w:
        res["w"] = out_w if out_w is not None else torch.empty((B, S, n0), dtype=torch.complex64,
                                                               device=dev)
    if want_power:
        res["power"] = torch.empty((B, S, n0), dtype=torch.float32, device=dev)
    if want_sig:
        res["sig"] = torch.empty((B, S, n0), dtype=torch.float32, device=dev)
    mid, mpar = _mother_args(mother, f0)
    if mid != 0 and n0 > 16384:
        raise ValueError("non-Morlet mothers: series of at most 16384 samples")
    ws = _long_workspace(B, n0, S, 0, dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_cwt_mother", _ptr(x), x.stride(0), B, n0, _ptr(aff), _ptr(sc), S,
                  float(dt), mid, mpar, _ptr(ss), sig_ld, _ptr(res.get("w")),
                  _ptr(res.get("power")), _ptr(res.get("sig")), _ptr(ws), _stream(dev))
    return res


MAX_SAMPLES = 1 << 20  # longest row the engine transforms (include/wtmi.h)


def cwt_workspace_bytes(batch: int, n0: int, n_scales: int, pair: bool = False) -> int:
    """Scratch bytes of a CWT / XWT launch (0 up to 16384 samples per row)."""
    return int(_lib.call("wtmi_cwt_workspace_bytes", batch, n0, n_scales, int(pair)))


def _long_workspace(B, n0, S, pair, dev):
    if n0 > MAX_SAMPLES:
        raise ValueError(f"series of {n0} samples: the engine transforms at most {MAX_SAMPLES}")
    need = cwt_workspace_bytes(B, n0, S, bool(pair))
    return torch.empty(need, dtype=torch.uint8, device=dev) if need > 0 else None


def _pair_rows(x1, x2):
    x1 = _rows(x1, torch.float32)
    x2 = _rows(x2, torch.float32)
    if x1.shape != x2.shape:
        raise ValueError("x1 and x2 must have the same shape")
    if x1.stride(0) != x2.stride(0):
        x1, x2 = x1.contiguous(), x2.contiguous()
    return x1, x2


def xwt_morlet(x1: torch.Tensor, x2: torch.Tensor, scales, dt: float, f0: float = 6.0, *,
               affine1=None, affine2=None, sig_scale=None, want_w12=False, want_power=False,
               want_sig=False, want_uv=False, mother=None):
    """Cross-wavelet outputs of row pairs: any of w12 (complex64), power, sig, u, v.
    sig_scale: [S] or per-pair [B, S] (1 / signif).  mother: as cwt_morlet."""
    x1, x2 = _pair_rows(x1, x2)
    B, n0 = x1.shape
    S = _n_scales(scales)
    sig_ld = _check_sig(sig_scale, B, S, want_sig)
    _check_affine(affine1, B, "affine1")
    _check_affine(affine2, B, "affine2")
    if not (want_w12 or want_power or want_sig or want_uv):
        raise ValueError("xwt_morlet: no output requested")
    dev = _check_dev(x1, x2, affine1, affine2)
    sc = _f64_dev(scales, dev)
    ss = _f64_dev(sig_scale, dev) if want_sig else None
    a1, a2 = _f64_arg(affine1, dev), _f64_arg(affine2, dev)
    shape = (B, S, n0)
    res = {}
    if want_w12:
        res["w12"] = torch.empty(shape, dtype=torch.complex64, device=dev)
    if want_power:
        res["power"] = torch.empty(shape, dtype=torch.float32, device=dev)
    if want_sig:
        res["sig"] = torch.empty(shape, dtype=torch.float32, device=dev)
    if want_uv:
        res["u"] = torch.empty(shape, dtype=torch.float32, device=dev)
        res["v"] = torch.empty(shape, dtype=torch.float32, device=dev)
    mid, mpar = _mother_args(mother, f0)
    if mid != 0 and n0 > 16384:
        raise ValueError("non-Morlet mothers: series of at most 16384 samples")
    ws = _long_workspace(B, n0, S, 1, dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_xwt_mother", _ptr(x1), _ptr(x2), x1.stride(0), B, n0, _ptr(a1), _ptr(a2),
                  _ptr(sc), S, float(dt), mid, mpar, _ptr(ss), sig_ld, _ptr(res.get("w12")),
                  _ptr(res.get("power")), _ptr(res.get("sig")), _ptr(res.get("u")),
                  _ptr(res.get("v")), _ptr(ws), _stream(dev))
    return res


def wct_workspace_bytes(batch: int, n0: int, n_scales: int) -> int:
    return int(_lib.call("wtmi_wct_workspace_bytes", batch, n0, n_scales))


def wct_morlet(x1: torch.Tensor, x2: torch.Tensor, scales, dt: float, f0: float = 6.0, *,
               boxcar: int, affine1=None, affine2=None, want_uv: bool = True,
               want_power: bool = False, want_phase: bool = False,
               workspace: Optional[torch.Tensor] = None, normalize: bool = False):
    """Wavelet coherence of row pairs; returns dict coh [B,S,n0] (+ u, v, power =
    |W1 W2*|^2, phase = angle(W1 W2*)).  normalize: pycwt's (y - mean) / std of each series,
    done inside the transform (wtmi_wct_morlet_norm; rows of 9..16384 samples, affine must
    then be None)."""
    x1, x2 = _pair_rows(x1, x2)
    B, n0 = x1.shape
    S = _n_scales(scales)
    _check_affine(affine1, B, "affine1")
    _check_affine(affine2, B, "affine2")
    if n0 > MAX_SAMPLES:
        raise ValueError(f"series of {n0} samples: the engine transforms at most {MAX_SAMPLES}")
    if int(boxcar) < 1:
        raise ValueError("boxcar must be >= 1")
    need = wct_workspace_bytes(B, n0, S)
    if workspace is not None and (not isinstance(workspace, torch.Tensor) or
                                  workspace.dtype != torch.uint8 or not workspace.is_contiguous()
                                  or workspace.numel() < need):
        raise ValueError(f"workspace must be a contiguous uint8 tensor of >= {need} bytes")
    dev = _check_dev(x1, x2, affine1, affine2, workspace)
    sc = _f64_dev(scales, dev)
    if workspace is None:
        workspace = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    shape = (B, S, n0)
    res = {"coh": torch.empty(shape, dtype=torch.float32, device=dev)}
    if want_power:
        res["power"] = torch.empty(shape, dtype=torch.float32, device=dev)
    if want_phase:
        res["phase"] = torch.empty(shape, dtype=torch.float32, device=dev)
    if want_uv:
        res["u"] = torch.empty(shape, dtype=torch.float32, device=dev)
        res["v"] = torch.empty(shape, dtype=torch.float32, device=dev)
    a1, a2 = _f64_arg(affine1, dev), _f64_arg(affine2, dev)
    if normalize and (a1 is not None or a2 is not None or not 8 < n0 <= 16384):
        raise ValueError("normalize=True: rows of 9..16384 samples and no affine coefficients")
    with torch.cuda.device(dev):
        if normalize:
            _lib.call("wtmi_wct_morlet_norm", _ptr(x1), _ptr(x2), x1.stride(0), B, n0, _ptr(sc), S,
                      float(dt), float(f0), int(boxcar), _ptr(workspace), _ptr(res["coh"]),
                      _ptr(res.get("power")), _ptr(res.get("phase")), _ptr(res.get("u")),
                      _ptr(res.get("v")), _stream(dev))
        else:
            _lib.call("wtmi_wct_morlet", _ptr(x1), _ptr(x2), x1.stride(0), B, n0, _ptr(a1), _ptr(a2),
                      _ptr(sc), S, float(dt), float(f0), int(boxcar), _ptr(workspace),
                      _ptr(res["coh"]), _ptr(res.get("power")), _ptr(res.get("phase")),
                      _ptr(res.get("u")), _ptr(res.get("v")), _stream(dev))
    return res


NOISE_MODES = ("pycwt", "red")


def rednoise(count: int, n: int, g: float, seed: int, *, first_series: int = 0,
             device=None, out: Optional[torch.Tensor] = None, noise: str = "pycwt") -> torch.Tensor:
    """[count, n] float32 Monte-Carlo noise, pycwt helpers.rednoise(n, g, 1) per row, drawn on
    the GPU from Philox4x32-10 stream (seed, first_series + row).  noise="pycwt" (default) is
    pycwt's literal behaviour: its lfilter runs along the length-1 axis of randn(n + tau, 1),
    so the rows are white normals (g sets only the burn-in tau); noise="red" applies the AR(1)
    filter the MATLAB original intends."""
    if noise not in NOISE_MODES:
        raise ValueError(f"noise must be one of {NOISE_MODES}, got {noise!r}")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if out is None:
        out = torch.empty((count, n), dtype=torch.float32, device=dev)
    _check_dev(out)
    with torch.cuda.device(out.device):
        _lib.call("wtmi_rednoise", _ptr(out), out.stride(0), count, n, float(g), int(noise == "red"),
                  C.c_ulonglong(int(seed) & ((1 << 64) - 1)), C.c_ulonglong(int(first_series)),
                  _stream(out.device))
    return out


def wct_side_streams() -> int:
    """Side streams the full-row WCT has created in this process (the pool's size)."""
    return int(_lib.load().wtmi_wct_side_streams())


def coherence_histogram(coh: torch.Tensor, t_lo: torch.Tensor, t_hi: torch.Tensor,
                        n_hist_scales: int, nbins: int = 1000,
                        hist: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Accumulate floor(coh * nbins) counts of coh [B, S, n0] over t in [t_lo[s], t_hi[s])
    for s < n_hist_scales into hist [n_hist_scales, nbins] (int32 view of uint32)."""
    if coh.dim() == 2:
        coh = coh.unsqueeze(0)
    coh = coh.to(torch.float32).contiguous()
    dev = _check_dev(coh)
    B, S, n0 = coh.shape
    lo = t_lo.to(device=dev, dtype=torch.int32).contiguous()
    hi = t_hi.to(device=dev, dtype=torch.int32).contiguous()
    if lo.numel() < n_hist_scales or hi.numel() < n_hist_scales:
        raise ValueError("t_lo / t_hi need one entry per histogram scale")
    if hist is None:
        hist = torch.zeros((n_hist_scales, nbins), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_coherence_histogram", _ptr(coh), B, n0, S, _ptr(lo), _ptr(hi),
                  int(n_hist_scales), int(nbins), _ptr(hist), _stream(dev))
    return hist


def coherence_quantile(hist: torch.Tensor, n_scales: int, level: float) -> torch.Tensor:
    """Per-scale level of the Monte-Carlo counter hist [>= n_scales, nbins] (int32 view of
    uint32) at `level` (wct_significance's quantile step, on the device): float64 [n_scales]."""
    dev = _check_dev(hist)
    hist = hist.contiguous()
    if hist.dim() != 2 or hist.shape[0] < n_scales:
        raise ValueError("hist must be [>= n_scales, nbins]")
    out = torch.empty(max(n_scales, 1), dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_coherence_quantile", _ptr(hist), int(n_scales), int(hist.shape[1]), float(level),
                  _ptr(out), _stream(dev))
    return out[:n_scales]


# -------------------------------------------------------------------------- MODWT
def _taps(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _out(out, shape, dev):
    if out is None:
        return torch.empty(shape, dtype=torch.float32, device=dev)
    if tuple(out.shape) != tuple(shape) or out.dtype != torch.float32 or not out.is_contiguous() \
            or out.device != dev:
        raise ValueError(f"out must be a contiguous float32 tensor of shape {tuple(shape)} on {dev}")
    return out


def modwt(x: torch.Tensor, dec_lo, dec_hi, level: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[B, n] float32 -> [B, level + 1, n] rows [W_1 .. W_J, V_J]."""
    x = _rows(x, torch.float32)
    dev = _check_dev(x)
    B, n = x.shape
    lo, hi = _taps(dec_lo), _taps(dec_hi)
    w = _out(out, (B, level + 1, n), dev)
    ws = _scratch(_lib.call("wtmi_modwt_workspace_bytes", B, n, int(level)), dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_modwt", _ptr(x), x.stride(0), B, n, lo.ctypes.data_as(VP),
                  hi.ctypes.data_as(VP), lo.size, int(level), _ptr(w), _ptr(ws), _stream(dev))
    return w


def _scratch(nbytes: int, dev):
    """Device scratch of a long-series launch (None when the call needs none)."""
    if nbytes < 0:
        raise ValueError("invalid geometry")
    return torch.empty(nbytes, dtype=torch.uint8, device=dev) if nbytes > 0 else None


def imodwt(w: torch.Tensor, dec_lo, dec_hi, keep_mask: Optional[int] = None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[B, J + 1, n] -> [B, n]; rows with a clear bit in keep_mask count as zero."""
    if w.dim() == 2:
        w = w.unsqueeze(0)
    w = w.to(torch.float32).contiguous()
    dev = _check_dev(w)
    B, R, n = w.shape
    lo, hi = _taps(dec_lo), _taps(dec_hi)
    keep = (1 << 64) - 1 if keep_mask is None else int(keep_mask)
    x = _out(out, (B, n), dev)
    ws = _scratch(_lib.call("wtmi_modwt_workspace_bytes", B, n, R - 1), dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_imodwt", _ptr(w), B, n, lo.ctypes.data_as(VP), hi.ctypes.data_as(VP),
                  lo.size, R - 1, C.c_ulonglong(keep), _ptr(x), x.stride(0), _ptr(ws), _stream(dev))
    return x


# ---------------------------------------------------------------------------- DWT
def dwt_lengths(n: int, n_taps: int, level: int) -> list:
    lens = (C.c_longlong * (level + 1))()
    total = _lib.call("wtmi_dwt_lengths", n, n_taps, level, C.cast(lens, VP))
    if total < 0:
        raise ValueError("invalid DWT geometry")
    return list(lens)


def wavedec(x: torch.Tensor, dec_lo, dec_hi, level: int):
    """Returns (coeffs [B, total] float32 in pywt order, lens)."""
    x = _rows(x, torch.float32)
    dev = _check_dev(x)
    B, n = x.shape
    lo, hi = _taps(dec_lo), _taps(dec_hi)
    lens = dwt_lengths(n, lo.size, level)
    coeffs = torch.empty((B, sum(lens)), dtype=torch.float32, device=dev)
    ws = _scratch(_lib.call("wtmi_dwt_workspace_bytes", B, n, lo.size, 1), dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_wavedec", _ptr(x), x.stride(0), B, n, lo.ctypes.data_as(VP),
                  hi.ctypes.data_as(VP), lo.size, int(level), _ptr(coeffs), _ptr(ws), _stream(dev))
    return coeffs, lens


def waverec(coeffs: torch.Tensor, n: int, rec_lo, rec_hi, level: int,
            keep_masks: Sequence[int]) -> torch.Tensor:
    """[B, total] -> [B, V, out_len]: one reconstruction per keep mask (bit k keeps
    list entry k of [cA_J, cD_J, ..., cD_1])."""
    if coeffs.dim() == 1:
        coeffs = coeffs.unsqueeze(0)
    coeffs = coeffs.to(torch.float32).contiguous()
    dev = _check_dev(coeffs)
    lo, hi = _taps(rec_lo), _taps(rec_hi)
    lens = dwt_lengths(n, lo.size, level)
    out_len = 2 * lens[-1] - lo.size + 2 if level > 0 else n
    masks = torch.as_tensor(np.asarray([int(m) & ((1 << 64) - 1) for m in keep_masks],
                                       dtype=np.uint64).view(np.int64), device=dev)
    B = coeffs.shape[0]
    out = torch.empty((B, len(keep_masks), out_len), dtype=torch.float32, device=dev)
    if level == 0 and n > 16384:  # nothing to invert: the kept cA_0 is the series
        keep = torch.tensor([float(int(m) & 1) for m in keep_masks], device=dev)
        return coeffs[:, None, :n] * keep[None, :, None]
    ws = _scratch(_lib.call("wtmi_dwt_workspace_bytes", B, n, lo.size, len(keep_masks)), dev)
    with torch.cuda.device(dev):
        _lib.call("wtmi_waverec", _ptr(coeffs), B, n, lo.ctypes.data_as(VP),
                  hi.ctypes.data_as(VP), lo.size, int(level), _ptr(masks), len(keep_masks),
                  _ptr(out), out_len, _ptr(ws), _stream(dev))
    return out


# ------------------------------------------------------------ torch custom ops
# torch.ops.wtmi.* wrappers over the same HIP kernels (CUDA/ROCm dispatch only: a
# CPU tensor has no kernel and raises).  Filter taps travel as host float64 tensors.
def _register():
    lib = torch.library

    @lib.custom_op("wtmi::cwt", mutates_args=())
    def _cwt(x: torch.Tensor, scales: torch.Tensor, dt: float, f0: float) -> torch.Tensor:
        return cwt_morlet(x, scales, dt, f0)["w"]

    @_cwt.register_fake
    def _(x, scales, dt, f0):
        return x.new_empty((x.shape[0] if x.dim() == 2 else 1, scales.numel(), x.shape[-1]),
                           dtype=torch.complex64)

    @lib.custom_op("wtmi::cwt_power", mutates_args=())
    def _cwt_power(x: torch.Tensor, scales: torch.Tensor, dt: float, f0: float) -> torch.Tensor:
        return cwt_morlet(x, scales, dt, f0, want_w=False, want_power=True)["power"]

    @_cwt_power.register_fake
    def _(x, scales, dt, f0):
        return x.new_empty((x.shape[0] if x.dim() == 2 else 1, scales.numel(), x.shape[-1]),
                           dtype=torch.float32)

    @lib.custom_op("wtmi::wct", mutates_args=())
    def _wct(x1: torch.Tensor, x2: torch.Tensor, scales: torch.Tensor, dt: float, f0: float,
             boxcar: int) -> torch.Tensor:
        return wct_morlet(x1, x2, scales, dt, f0, boxcar=boxcar, want_uv=False)["coh"]

    @_wct.register_fake
    def _(x1, x2, scales, dt, f0, boxcar):
        return x1.new_empty((x1.shape[0] if x1.dim() == 2 else 1, scales.numel(), x1.shape[-1]),
                            dtype=torch.float32)

    @lib.custom_op("wtmi::modwt", mutates_args=())
    def _modwt(x: torch.Tensor, dec_lo: torch.Tensor, dec_hi: torch.Tensor, level: int
               ) -> torch.Tensor:
        return modwt(x, dec_lo.cpu().numpy(), dec_hi.cpu().numpy(), level)

    @_modwt.register_fake
    def _(x, dec_lo, dec_hi, level):
        return x.new_empty((x.shape[0] if x.dim() == 2 else 1, level + 1, x.shape[-1]),
                           dtype=torch.float32)

    @lib.custom_op("wtmi::imodwt", mutates_args=())
    def _imodwt(w: torch.Tensor, dec_lo: torch.Tensor, dec_hi: torch.Tensor) -> torch.Tensor:
        return imodwt(w, dec_lo.cpu().numpy(), dec_hi.cpu().numpy())

    @_imodwt.register_fake
    def _(w, dec_lo, dec_hi):
        return w.new_empty((w.shape[0] if w.dim() == 3 else 1, w.shape[-1]), dtype=torch.float32)

    def _bs(x, scales, dtype):
        return x.new_empty((x.shape[0] if x.dim() == 2 else 1, scales.numel(), x.shape[-1]),
                           dtype=dtype)

    @lib.custom_op("wtmi::xwt", mutates_args=())
    def _xwt(x1: torch.Tensor, x2: torch.Tensor, scales: torch.Tensor, dt: float, f0: float
             ) -> torch.Tensor:
        """W1 W2* (complex64) of row pairs (pycwt.xwt before normalisation)."""
        return xwt_morlet(x1, x2, scales, dt, f0, want_w12=True)["w12"]

    @_xwt.register_fake
    def _(x1, x2, scales, dt, f0):
        return _bs(x1, scales, torch.complex64)

    @lib.custom_op("wtmi::xwt_power", mutates_args=())
    def _xwt_power(x1: torch.Tensor, x2: torch.Tensor, scales: torch.Tensor, dt: float, f0: float
                   ) -> torch.Tensor:
        return xwt_morlet(x1, x2, scales, dt, f0, want_power=True)["power"]

    @_xwt_power.register_fake
    def _(x1, x2, scales, dt, f0):
        return _bs(x1, scales, torch.float32)

    @lib.custom_op("wtmi::dwt", mutates_args=())
    def _dwt(x: torch.Tensor, dec_lo: torch.Tensor, dec_hi: torch.Tensor, level: int
             ) -> torch.Tensor:
        """pywt.wavedec (mode symmetric), coefficient lists back-to-back: [B, total]."""
        return wavedec(x, dec_lo.cpu().numpy(), dec_hi.cpu().numpy(), level)[0]

    @_dwt.register_fake
    def _(x, dec_lo, dec_hi, level):
        total = sum(dwt_lengths(x.shape[-1], dec_lo.numel(), level))
        return x.new_empty((x.shape[0] if x.dim() == 2 else 1, total), dtype=torch.float32)

    @lib.custom_op("wtmi::idwt", mutates_args=())
    def _idwt(coeffs: torch.Tensor, n: int, rec_lo: torch.Tensor, rec_hi: torch.Tensor,
              level: int) -> torch.Tensor:
        """pywt.waverec of back-to-back coefficient lists: [B, out_len]."""
        full = (1 << (level + 1)) - 1
        return waverec(coeffs, n, rec_lo.cpu().numpy(), rec_hi.cpu().numpy(), level, [full])[:, 0]

    @_idwt.register_fake
    def _(coeffs, n, rec_lo, rec_hi, level):
        lens = dwt_lengths(n, rec_lo.numel(), level)
        out_len = 2 * lens[-1] - rec_lo.numel() + 2 if level > 0 else n
        return coeffs.new_empty((coeffs.shape[0] if coeffs.dim() == 2 else 1, out_len),
                                dtype=torch.float32)

    @lib.custom_op("wtmi::series_stats", mutates_args=())
    def _series_stats(x: torch.Tensor) -> torch.Tensor:
        """[B, 8] float64: mean, std, detrend slope, intercept, lag-0 / lag-1 covariance, n, 0."""
        return series_moments(x)

    @_series_stats.register_fake
    def _(x):
        return x.new_empty((x.shape[0] if x.dim() == 2 else 1, 8), dtype=torch.float64)


try:
    torch.ops.wtmi.cwt  # already registered (module reloaded)
except (AttributeError, RuntimeError):
    _register()
