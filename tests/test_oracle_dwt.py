"""Pin the DWT oracle against PyWavelets 1.1.1 outputs and the reference's own helpers."""

import numpy as np

from oracle import dwt_spec as ds
from oracle import glue_spec as gs


def _case(g, i):
    nlev = int(g[f"c{i}_nlev"])
    lvl = int(g[f"c{i}_level"])
    return (g[f"c{i}_x"], str(g[f"c{i}_wavelet"]), None if lvl < 0 else lvl,
            [g[f"c{i}_coef{k}"] for k in range(nlev)])


def test_wavedec_waverec_match_pywt(dwt_golden, pywt_filters):
    g = dwt_golden
    for i in range(int(g["ncases"])):
        x, wname, level, coeffs = _case(g, i)
        f = pywt_filters[wname]
        got = ds.wavedec(x, f["dec_lo"], f["dec_hi"], level)
        assert [c.size for c in got] == [c.size for c in coeffs], (i, wname)
        for a, b in zip(got, coeffs):
            np.testing.assert_allclose(a, b, rtol=0, atol=1e-12 * max(1, np.abs(b).max()))
        rec = ds.waverec(coeffs, f["rec_lo"], f["rec_hi"])
        ref = g[f"c{i}_rec"]
        assert rec.size == ref.size
        np.testing.assert_allclose(rec, ref, rtol=0, atol=1e-11 * max(1, np.abs(ref).max()))
        assert ds.dwt_max_level(x.size, len(f["dec_lo"])) == int(g[f"c{i}_maxlevel"])


def test_smooth_and_components_match_reference(dwt_golden, pywt_filters):
    g = dwt_golden
    f = pywt_filters["db4"]
    seen = 0
    for i in range(int(g["ncases"])):
        if f"c{i}_comp0" not in g:
            continue
        seen += 1
        x, wname, level, coeffs = _case(g, i)
        levels = len(coeffs) - 1
        sm = gs.dwt_smooth_signal(coeffs, levels, x, f["rec_lo"], f["rec_hi"])
        for lvl in range(1, levels + 1):
            ref = g[f"c{i}_smooth{lvl}"]
            assert sm[lvl]["signal"].size == ref.size
            np.testing.assert_allclose(sm[lvl]["signal"], ref, atol=1e-10, rtol=0)
        for lvl in range(len(coeffs)):
            comp = gs.reconstruct_signal_component(coeffs, lvl, f["rec_lo"], f["rec_hi"])
            np.testing.assert_allclose(comp, g[f"c{i}_comp{lvl}"], atol=1e-10, rtol=0)
    assert seen >= 3


def test_filters_are_orthogonal_banks(pywt_filters):
    for name, f in pywt_filters.items():
        lo = np.asarray(f["dec_lo"])
        assert np.isclose(lo.sum(), np.sqrt(2), atol=1e-9), name
        assert np.isclose((lo ** 2).sum(), 1.0, atol=1e-9), name
        k = np.arange(lo.size)
        np.testing.assert_array_equal(np.asarray(f["rec_lo"]), lo[::-1])
        np.testing.assert_array_equal(np.asarray(f["rec_hi"]), ((-1.0) ** k) * lo)
        np.testing.assert_array_equal(np.asarray(f["dec_hi"]), (((-1.0) ** k) * lo)[::-1])
