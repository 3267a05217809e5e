"""Generate the golden fixtures that pin the CPU oracle.

Run in the BUILD container (it reads /root/reference, which does not exist on the
GPU box) with the conda interpreter that has PyWavelets 1.1.1:

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

Outputs (small, committed):
  tests/golden/modwt_golden.npz   outputs of the reference's OWN src/modwt.py
                                   functions (modwt, imodwt, modwtmra, smooth_signal)
  tests/golden/dwt_golden.npz     outputs of PyWavelets 1.1.1 wavedec/waverec and of
                                   the reference's own src/dwt.py helpers
  tests/golden/pywt_filters.json  orthogonal filter banks from PyWavelets 1.1.1

How the reference code is executed: the pure functions are extracted from the
source text with ``ast`` (a plain ``import src.modwt`` fails here: its module
imports pycwt/statsmodels/streamlit chains) and executed in a namespace holding
only numpy, pywt and scipy.ndimage.convolve1d.  Nothing from the reference is
written into the repository except these input/output vectors.
"""

import ast
import json
import os
import sys
from dataclasses import dataclass, field
from typing import Dict, Type

import numpy as np
import pywt
from scipy.ndimage import convolve1d

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


class _NullLog:
    def __getattr__(self, _):
        return lambda *a, **k: None


def load_functions(path, names):
    """The named reference definitions, executed only after each segment's SHA-256 matches
    its pin (scripts/refpin.py, scripts/refpins.json)."""
    sys.path.insert(0, os.path.join(HERE, "..", "..", "scripts"))
    import refpin
    mod = refpin.pinned_module(REF, os.path.relpath(path, REF), sorted(names))
    ns = {"np": np, "npt": np.typing if hasattr(np, "typing") else None,
          "pywt": pywt, "convolve1d": convolve1d, "dataclass": dataclass,
          "field": field, "Dict": Dict, "Type": Type, "logger": _NullLog(),
          "print": lambda *a, **k: None}
    import numpy.typing  # noqa: F401
    ns["npt"] = np.typing
    exec(compile(mod, path, "exec"), ns)
    return ns


def make_modwt():
    ns = load_functions(os.path.join(REF, "src/modwt.py"),
                        {"upArrow_op", "period_list", "circular_convolve_mra",
                         "circular_convolve_d", "circular_convolve_s", "modwt",
                         "imodwt", "modwtmra", "smooth_signal"})
    rng = np.random.default_rng(20251031)
    cases = [(64, j, "f8") for j in range(1, 7)] + [
        (100, 5, "f8"), (16, 8, "f8"), (7, 3, "f8"), (1333, 6, "f8"),
        (1333, 6, "f4"), (4096, 10, "f4"), (4096, 10, "f8"), (256, 4, "f4"),
    ]
    out = {}
    for idx, (n, J, dt) in enumerate(cases):
        x = rng.standard_normal(n).cumsum() * 0.1 + rng.standard_normal(n)
        x = x.astype(dt)
        w = ns["modwt"](x, "db4", J)
        out[f"c{idx}_x"] = x
        out[f"c{idx}_w"] = w
        out[f"c{idx}_J"] = np.int64(J)
        out[f"c{idx}_inv"] = ns["imodwt"](w, "db4")
        # inverse of a NON-range input (adjoint check) on the small cases
        if n <= 1333:
            wr = rng.standard_normal(w.shape).astype(dt)
            out[f"c{idx}_wrand"] = wr
            out[f"c{idx}_invrand"] = ns["imodwt"](wr, "db4")
        if n in (64, 100, 1333) and dt == "f8":
            out[f"c{idx}_mra"] = ns["modwtmra"](w, "db4")
            sm = ns["smooth_signal"](w, "db4", J)
            for lvl, d in sm.items():
                out[f"c{idx}_smooth{lvl}"] = d["signal"]
    out["ncases"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(HERE, "modwt_golden.npz"), **out)
    print("modwt cases", len(cases))


def make_dwt():
    ns = load_functions(os.path.join(REF, "src/dwt.py"),
                        {"ResultsFromDWT", "trim_signal", "reconstruct_signal_component"})
    rng = np.random.default_rng(1914)
    cases = [(3, "db4", None), (5, "db4", None), (8, "db4", None), (9, "db4", 1),
             (13, "db4", None), (101, "db4", None), (101, "db2", 3), (565, "db4", None),
             (1333, "db4", None), (1334, "db4", 5), (16384, "db4", None),
             (50, "haar", None), (64, "sym5", 2)]
    out = {}
    for idx, (n, wname, level) in enumerate(cases):
        w = pywt.Wavelet(wname)
        x = rng.standard_normal(n).cumsum()
        coeffs = pywt.wavedec(x, w, level=level)
        out[f"c{idx}_x"] = x
        out[f"c{idx}_wavelet"] = np.array(wname)
        out[f"c{idx}_level"] = np.int64(-1 if level is None else level)
        out[f"c{idx}_nlev"] = np.int64(len(coeffs))
        for k, c in enumerate(coeffs):
            out[f"c{idx}_coef{k}"] = c
        out[f"c{idx}_rec"] = pywt.waverec(coeffs, w)
        out[f"c{idx}_maxlevel"] = np.int64(pywt.dwt_max_level(n, w.dec_len))
        if n in (101, 565, 1333, 1334) and wname == "db4":
            levels = len(coeffs) - 1
            res = ns["ResultsFromDWT"](coeffs, levels)
            res.smooth_signal(x, w)
            for lvl, d in res.smoothed_signal_dict.items():
                out[f"c{idx}_smooth{lvl}"] = d["signal"]
            for lvl in range(len(coeffs)):
                out[f"c{idx}_comp{lvl}"] = ns["reconstruct_signal_component"](
                    list(coeffs), w, lvl)
    out["ncases"] = np.int64(len(cases))
    np.savez_compressed(os.path.join(HERE, "dwt_golden.npz"), **out)
    print("dwt cases", len(cases))


def make_filters():
    names = ["haar"] + [f"db{i}" for i in range(1, 21)] + \
            [f"sym{i}" for i in range(2, 21)] + [f"coif{i}" for i in range(1, 18)]
    table = {}
    for nm in names:
        w = pywt.Wavelet(nm)
        table[nm] = {"dec_lo": list(map(float, w.dec_lo)), "dec_hi": list(map(float, w.dec_hi)),
                     "rec_lo": list(map(float, w.rec_lo)), "rec_hi": list(map(float, w.rec_hi))}
    with open(os.path.join(HERE, "pywt_filters.json"), "w") as f:
        json.dump({"pywt_version": pywt.__version__, "filters": table}, f)
    print("filters", len(table))


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference tree not found; run in the build container")
    make_filters()
    make_modwt()
    make_dwt()
