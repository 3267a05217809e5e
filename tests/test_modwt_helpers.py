"""src.modwt's host-side helpers (upArrow_op, period_list, circular_convolve_{d,s,mra})
against the reference's own outputs (tests/golden/modwt_golden.npz), CPU only.

The reference builds modwt / imodwt / modwtmra from these helpers (src/modwt.py:126-194);
composing the repo's helpers the same way must reproduce the golden vectors (fp64 cases to
1e-12 relative, fp32 cases to fp32 resolution).  The engine's own modwt/imodwt are the GPU
kernels (tests/test_gpu_modwt_dwt.py); these helpers only keep the module surface whole.
"""

import numpy as np
import pytest

from src import modwt as M


def _ncases(g):
    return int(g["ncases"])


def _tol(x):
    return 1e-12 if x.dtype == np.float64 else 2e-6


def test_up_arrow_and_period_list():
    assert M.upArrow_op([1, 2, 3], 0) == [1]
    np.testing.assert_array_equal(M.upArrow_op([1, 2, 3], 1), [1, 2, 3])
    np.testing.assert_array_equal(M.upArrow_op([1, 2, 3], 3), [1, 0, 0, 0, 2, 0, 0, 0, 3])
    np.testing.assert_array_equal(M.period_list([1, 2, 3], 5), [1, 2, 3, 0, 0])
    np.testing.assert_array_equal(M.period_list(np.arange(1, 8), 3), [1 + 4 + 7, 2 + 5, 3 + 6])
    np.testing.assert_array_equal(M.period_list([1, 2, 3], 3), [1, 2, 3])


def test_cascades_from_helpers_match_reference_golden(modwt_golden, db4):
    g = modwt_golden
    h_t = np.asarray(db4["dec_hi"]) / np.sqrt(2)
    g_t = np.asarray(db4["dec_lo"]) / np.sqrt(2)
    for c in range(_ncases(g)):
        x, J = g[f"c{c}_x"], int(g[f"c{c}_J"])
        rows, v = [], x
        for j in range(1, J + 1):
            rows.append(M.circular_convolve_d(h_t, v, j))
            v = M.circular_convolve_d(g_t, v, j)
        rows.append(v)
        w = np.vstack(rows)
        ref = g[f"c{c}_w"]
        assert w.dtype == ref.dtype
        assert np.abs(w - ref).max() <= _tol(x) * np.abs(ref).max(), c
        vj = ref[-1]
        for j in range(J, 0, -1):
            vj = M.circular_convolve_s(h_t, g_t, ref[j - 1], vj, j)
        inv = g[f"c{c}_inv"]
        assert np.abs(vj - inv).max() <= _tol(x) * np.abs(inv).max(), c


def test_mra_from_helpers_matches_reference_golden(modwt_golden, db4):
    """The reference's dense-filter MRA (src/modwt.py:163-194) rebuilt from the helpers."""
    g = modwt_golden
    h, gl = np.asarray(db4["dec_hi"]), np.asarray(db4["dec_lo"])
    seen = 0
    for c in range(_ncases(g)):
        if f"c{c}_mra" not in g:
            continue
        w = g[f"c{c}_w"]
        level, N = w.shape[0] - 1, w.shape[1]
        D, gpart = [], [1]
        for j in range(level):
            gpart = np.convolve(gpart, M.upArrow_op(gl, j))
            hj = np.convolve(gpart, M.upArrow_op(h, j + 1)) / 2 ** ((j + 1) / 2.0)
            if j == 0:
                hj = h / np.sqrt(2)
            D.append(M.circular_convolve_mra(M.period_list(hj, N), w[j]))
        gj = np.convolve(gpart, M.upArrow_op(gl, level)) / 2 ** (level / 2.0)
        D.append(M.circular_convolve_mra(M.period_list(gj, N), w[-1]))
        ref = g[f"c{c}_mra"]
        assert np.abs(np.vstack(D) - ref).max() <= 1e-11 * np.abs(ref).max(), c
        seen += 1
    assert seen >= 3


def test_time_scale_regression_needs_statsmodels():
    try:
        import statsmodels  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            M.time_scale_regression([np.ones(4)], [np.ones(4)], 0)
    else:  # pragma: no cover - statsmodels is absent from this image
        M.time_scale_regression([np.arange(8.0)] * 2, [np.arange(8.0) * 2] * 2, 1)
