"""Pin the MODWT oracle against vectors produced by the reference's own src/modwt.py."""

import numpy as np
import pytest

from oracle import modwt_spec as ms


def _cases(g):
    for i in range(int(g["ncases"])):
        yield i, g[f"c{i}_x"], g[f"c{i}_w"], int(g[f"c{i}_J"])


def test_modwt_matches_reference_bitwise(modwt_golden, db4):
    for i, x, w, J in _cases(modwt_golden):
        got = ms.modwt(x, db4["dec_lo"], db4["dec_hi"], J)
        assert got.shape == w.shape == (J + 1, x.size)
        assert got.dtype == w.dtype, i
        # same algorithm, same scipy primitive -> bitwise identical (probe C.5)
        np.testing.assert_array_equal(got, w, err_msg=f"case {i}")


def test_imodwt_matches_reference(modwt_golden, db4):
    g = modwt_golden
    for i, x, w, J in _cases(g):
        inv = ms.imodwt(w, db4["dec_lo"], db4["dec_hi"])
        np.testing.assert_array_equal(inv, g[f"c{i}_inv"])
        if f"c{i}_wrand" in g:
            inv = ms.imodwt(g[f"c{i}_wrand"], db4["dec_lo"], db4["dec_hi"])
            np.testing.assert_array_equal(inv, g[f"c{i}_invrand"])


def test_direct_form_equals_reference(modwt_golden, db4):
    for i, x, w, J in _cases(modwt_golden):
        got = ms.modwt_direct(x, db4["dec_lo"], db4["dec_hi"], J)
        tol = 2e-6 if x.dtype == np.float32 else 1e-12
        scale = np.abs(w).max()
        assert np.abs(got - w).max() <= tol * scale * (J + 1), i
        inv = ms.imodwt_direct(w, db4["dec_lo"], db4["dec_hi"])
        ref = modwt_golden[f"c{i}_inv"]
        assert np.abs(inv - ref).max() <= tol * np.abs(ref).max() * (J + 1), i


def test_round_trip_and_energy(modwt_golden, db4):
    for i, x, w, J in _cases(modwt_golden):
        if x.dtype != np.float64:
            continue
        inv = ms.imodwt(w, db4["dec_lo"], db4["dec_hi"])
        assert np.abs(inv - x).max() < 1e-10
        assert np.isclose((w ** 2).sum(), (x ** 2).sum(), rtol=1e-10)


def test_mra_and_smooth(modwt_golden, db4):
    g = modwt_golden
    for i, x, w, J in _cases(g):
        if f"c{i}_mra" not in g:
            continue
        mra = ms.modwtmra(w, db4["dec_lo"], db4["dec_hi"])
        ref = g[f"c{i}_mra"]
        assert np.abs(mra - ref).max() < 1e-12 * max(1.0, np.abs(ref).max())
        np.testing.assert_allclose(mra.sum(axis=0), x, atol=1e-10)
        sm = ms.smooth_signal(w, db4["dec_lo"], db4["dec_hi"], J)
        for lvl in range(1, J + 1):
            np.testing.assert_allclose(sm[lvl]["signal"], g[f"c{i}_smooth{lvl}"],
                                       atol=1e-12, rtol=0)
