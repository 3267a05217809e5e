"""Non-Morlet mothers of the reference's MOTHER_DICT (src/xwt.py:29-34, src/wct.py:36-41,
constants/results_configs.py:53-58) through the CWT / XWT kernels (mother ids 1, 2 of
include/wtmi.h) against the oracle's restatement of pycwt's Paul / DOG (parity unpinned,
like every pycwt-derived value: pycwt is absent; pinned by tests/test_oracle_cwt.py's
known answers).  Tolerance: per (series, scale) row ||W - W_ref|| / ||W_ref|| <= 1e-5.
"""

import numpy as np
import pytest
import torch

from gpu_helpers import gate, red_series, row_relerr
from oracle import glue_spec as gs
from oracle import pycwt_spec as pc

pytestmark = pytest.mark.gpu
MOTHERS = [pc.Paul(4), pc.DOG(2), pc.MexicanHat(), pc.DOG(3), pc.Paul(6)]


def _rows_ok(W, ref, name="W", tol=1e-5):
    """Row error where the reference row carries energy (Paul rows at the largest scales of
    a short series can vanish to the fp64 floor); gated and printed by gpu_helpers.gate."""
    nrm = np.linalg.norm(ref, axis=-1)
    keep = nrm > 1e-6 * nrm.max()
    gate(name, row_relerr(W[keep], ref[keep]), tol)
    return True


@pytest.mark.parametrize("mother", MOTHERS, ids=lambda m: f"{m.name}{m.m}")
@pytest.mark.parametrize("n0", [5, 8, 100, 1333, 4096, 10000])
def test_cwt_other_mothers_match_oracle(mother, n0):
    from wtmi import transforms
    rng = np.random.default_rng(n0)
    x = red_series(rng, n0).astype(np.float64)
    J = 40 if n0 < 64 else -1
    W, sj, freqs, coi, _, _ = transforms.cwt(x.astype(np.float32).astype(np.float64), 1 / 12, 1 / 12,
                                             2 / 12, J, mother)
    rW, rsj, rfreqs, rcoi, _, _ = pc.cwt(x.astype(np.float32).astype(np.float64), 1 / 12, 1 / 12,
                                         2 / 12, J, mother)
    assert W.shape == rW.shape
    assert _rows_ok(W, rW)
    np.testing.assert_allclose(freqs, rfreqs, rtol=1e-12)
    np.testing.assert_allclose(coi, rcoi, rtol=1e-12)


@pytest.mark.parametrize("mother", MOTHERS[:3], ids=lambda m: f"{m.name}{m.m}")
def test_run_cwt_other_mothers(mother):
    """src.cwt.run_cwt with a pycwt-shaped mother object (duck-typed by class name and m):
    power, period, COI and the significance ratio (DOG: dofmin 1, chi2.ppf(0.95, 1))."""
    import src.cwt as cwt
    rng = np.random.default_rng(3)
    y = gs.standardize_series(red_series(rng, 700).astype(np.float64) + 0.01 * np.arange(700))
    t = np.arange(700).astype("datetime64[M]")
    d = cwt.DataForCWT(t, y, mother, cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS)
    r = cwt.run_cwt(d)
    p, period, sig, coi = gs.run_cwt(y, y.size, mother=mother)
    assert r.power.shape == p.shape
    assert _rows_ok(r.power, p, "run_cwt power")
    assert _rows_ok(r.significance_levels, sig, "run_cwt sig ratio")
    np.testing.assert_allclose(r.period, period, rtol=1e-12)
    np.testing.assert_allclose(r.coi, coi, rtol=1e-12)


@pytest.mark.parametrize("key", ["paul", "DOG", "mexicanhat"])
def test_run_xwt_other_mothers(key):
    """src.xwt.run_xwt with MOTHER_DICT[key] raises AttributeError, as the reference does in
    pycwt.wct (no Paul/DOG smooth), before any launch.  The engine's explicit alternative,
    run_xwt_batch(..., phase_without_smooth=True): power and significance ratio as pycwt.xwt
    + normalize_xwt_results; phase arrows from angle(W1 W2*) at dj = 1/12 (what pycwt.wct
    returns as aWCT)."""
    import src.xwt as xwt
    rng = np.random.default_rng(8)
    y1 = red_series(rng, 900).astype(np.float64)
    y2 = 0.6 * np.roll(y1, 4) + 0.8 * red_series(rng, 900)
    m = xwt.MOTHER_DICT[key]
    om = {"paul": pc.Paul(4), "DOG": pc.DOG(2), "mexicanhat": pc.MexicanHat()}[key]
    data = xwt.DataForXWT(y1, y2, m, xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
    with pytest.raises(AttributeError, match="smooth"):
        xwt.run_xwt(data)
    with pytest.raises(AttributeError, match="smooth"):
        xwt.run_xwt_batch([data])
    r = xwt.run_xwt_batch([data], phase_without_smooth=True)[0]
    W12, coi, freqs, signif = pc.xwt(y1, y2, dt=xwt.DT, dj=xwt.DJ, s0=xwt.S0, wavelet=om)
    period, power, sig95, coi_plot = gs.normalize_xwt_results(
        y1.size, W12, coi, np.log2(xwt.LEVELS[2]), freqs, signif)
    assert _rows_ok(r.power, power, "run_xwt power")
    assert _rows_ok(r.significance_levels, sig95, "run_xwt sig ratio")
    np.testing.assert_allclose(r.period, period, rtol=1e-12)
    np.testing.assert_allclose(r.coi, coi_plot, rtol=1e-12)
    n1 = (y1 - y1.mean()) / y1.std()
    n2 = (y2 - y2.mean()) / y2.std()
    Wp = pc.cwt(n1, xwt.DT, 1 / 12, xwt.S0, -1, om)[0] * pc.cwt(n2, xwt.DT, 1 / 12, xwt.S0, -1, om)[0].conj()
    u, v = gs.phase_uv(np.angle(Wp))
    mask = np.abs(Wp) > 1e-3 * np.abs(Wp).max()
    assert r.phase_diff_u.shape == u.shape
    np.testing.assert_allclose(r.phase_diff_u[mask], u[mask], atol=1e-4)
    np.testing.assert_allclose(r.phase_diff_v[mask], v[mask], atol=1e-4)


def test_wct_with_other_mother_raises_like_pycwt():
    import src.wct as wct
    rng = np.random.default_rng(1)
    y = red_series(rng, 300).astype(np.float64)
    d = wct.DataForWCT(y, y, wct.MOTHER_DICT["paul"], wct.DT, wct.DJ, wct.S0, wct.LEVELS)
    with pytest.raises(AttributeError, match="smooth"):
        wct.run_wct(d, calculate_signficance=False)


def test_torch_op_rejects_long_rows_for_other_mothers():
    from wtmi import ops
    x = torch.zeros((1, 20000), device="cuda")
    with pytest.raises(ValueError):
        ops.cwt_morlet(x, np.array([1.0]), 1 / 12, mother=pc.Paul(4))
