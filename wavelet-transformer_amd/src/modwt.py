"""Maximal-overlap DWT (reference: src/modwt.py:126-251).

``modwt`` / ``imodwt`` run the a-trous cascades on the GPU (``wtmi_modwt`` /
``wtmi_imodwt``: one workgroup per series, all J levels LDS-resident, only the L
non-zero taps per level).  ``modwtmra`` and ``smooth_signal`` are masked inverse
transforms (row j of the MRA = inverse of the isolated row j, probe C.8b).
Row order is the reference's ``[W_1 .. W_J, V_J]``; output dtype follows the input
dtype (float32 in -> float32 out, quirk B.11).
"""

from __future__ import annotations

import numpy as np

from wtmi import transforms
from wtmi.wavelets import Wavelet

MOTHER = Wavelet("db4")


def modwt(x, filters, level):
    """filters: 'db1', 'db2', 'haar', ... (or a filter-bank object); returns [level+1, N]."""
    return transforms.modwt(x, filters, level)


def imodwt(w, filters):
    """Inverse MODWT of rows [W_1 .. W_J, V_J]."""
    return transforms.imodwt(w, filters)


def modwtmra(w, filters):
    """Multiresolution analysis [D_1 .. D_J, S_J]."""
    w = np.asarray(w)
    return np.vstack([transforms.imodwt(w, filters, keep_mask=1 << j) for j in range(w.shape[0])])


def smooth_signal(modwt_coeffs, mother_wavelet, levels):
    """signal_dict[l]: inverse with detail rows 0..l-1 zeroed (src/modwt.py:232-251)."""
    signals_dict = {}
    c = np.asarray(modwt_coeffs)
    full = (1 << c.shape[0]) - 1
    for lvl in range(levels, 0, -1):
        print(f"s_{lvl} stored with key {lvl}")
        smooth_coeffs = c.copy()
        smooth_coeffs[:lvl] = 0
        keep = full & ~((1 << lvl) - 1)
        signals_dict[lvl] = {"coeffs": smooth_coeffs,
                             "signal": transforms.imodwt(c, mother_wavelet, keep_mask=keep)}
    return signals_dict
