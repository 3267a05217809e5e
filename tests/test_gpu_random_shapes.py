"""Seeded random-shape sweep of the HIP transforms against the oracle (r05).

The per-shape tests pin the configurations the reference and the bench use; this sweep draws
series lengths, scale resolutions, sampling steps, Morlet f0, batch sizes, filter banks and
levels at random (fixed seeds, so every run checks the same cases) to reach the launch paths
the hand-picked shapes do not: padded rows of every FFT size, rows past one workgroup (the
four-step long path), chunk counts, band-pruning regimes at several f0, odd lengths for the
MODWT and DWT.  Gates as SURVEY 8(d): CWT rows <= 1e-5 row-normwise (power too), WCT
coherence <= 1e-4 abs, MODWT rows <= 1e-5 normwise and round trip <= 1e-5 max|x|, DWT
coefficients <= 1e-5 of the row maximum.  The CWT / WCT oracle restates pycwt 0.4.0b0 (parity
unpinned: pycwt is absent), the MODWT / DWT oracle is pinned by the reference's own functions
and PyWavelets fixtures (tests/golden).
"""

import os

import numpy as np
import pytest
import torch

from gpu_helpers import gate, red_series, row_relerr
from oracle import dwt_spec as ds
from oracle import modwt_spec as ms
from oracle import pycwt_spec as pc

pytestmark = pytest.mark.gpu

# WTMI_RANDOM_SCALE = k draws k times as many cases per family (the first ones unchanged: the
# draws are sequential), for an extended sweep on demand; the default suite runs k = 1
SCALE = max(1, int(os.environ.get("WTMI_RANDOM_SCALE", "1")))


def _cwt_cases(seed=2025, count=24):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count * SCALE):
        n0 = int(np.exp(rng.uniform(np.log(9), np.log(40000))))
        dj = float(rng.choice([1 / 4, 1 / 6, 1 / 8, 1 / 12, 1 / 16, 1 / 24]))
        dt = float(rng.choice([1 / 12, 1.0, 0.25]))
        s0 = float(rng.choice([2.0, 3.0, 1.5])) * dt
        f0 = float(rng.choice([6.0, 6.0, 5.0, 8.0]))
        J = int(np.round(np.log2(n0 * dt / s0) / dj))
        J = max(1, min(J, 150 if n0 <= 16384 else 40))
        B = int(rng.integers(1, 4))
        out.append((i, n0, dj, dt, s0, f0, J, B))
    return out


@pytest.mark.parametrize("case", _cwt_cases(), ids=lambda c: f"cwt{c[0]}-n{c[1]}")
def test_random_cwt_matches_oracle(case):
    from wtmi import ops
    i, n0, dj, dt, s0, f0, J, B = case
    rng = np.random.default_rng(1000 + i)
    x = np.stack([red_series(rng, n0) for _ in range(B)])
    if B > 1:
        x[-1] += 30.0  # an offset: the removed-mean spectrum path
    sj = s0 * 2 ** (np.arange(J + 1) * dj)
    r = ops.cwt_morlet(torch.tensor(x, device="cuda"), sj, dt, f0, want_w=True, want_power=True)
    W, P = r["w"].cpu().numpy(), r["power"].cpu().numpy()
    for b in range(B):
        ref = pc.cwt(x[b].astype(np.float64), dt, dj, s0, J, pc.Morlet(f0))[0]
        assert W.shape[1:] == ref.shape
        gate(f"W[{b}]", row_relerr(W[b].astype(np.complex128), ref))
        gate(f"power[{b}]", row_relerr(P[b].astype(np.float64), np.abs(ref) ** 2))


def _wct_cases(seed=77, count=8):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count * SCALE):
        n0 = int(np.exp(rng.uniform(np.log(40), np.log(12000))))
        dj = float(rng.choice([1 / 4, 1 / 8, 1 / 12]))
        out.append((i, n0, dj))
    return out


@pytest.mark.parametrize("case", _wct_cases(), ids=lambda c: f"wct{c[0]}-n{c[1]}")
def test_random_wct_matches_oracle(case):
    from wtmi import transforms
    i, n0, dj = case
    rng = np.random.default_rng(2000 + i)
    y1 = red_series(rng, n0).astype(np.float64)
    y2 = 0.6 * np.roll(y1, 2) + 0.8 * red_series(rng, n0)
    coh, aw, coi, freq, _ = transforms.wct(y1, y2, 1 / 12, dj=dj, s0=2 / 12, J=-1, sig=False)
    rc, ra, rcoi, rfreq, _ = pc.wct(y1, y2, 1 / 12, dj=dj, s0=2 / 12, J=-1, sig=False)
    assert coh.shape == rc.shape
    gate("coherence abs", np.abs(coh - rc), 1e-4)
    W12 = (pc.cwt((y1 - y1.mean()) / y1.std(), 1 / 12, dj, 2 / 12, -1)[0]
           * pc.cwt((y2 - y2.mean()) / y2.std(), 1 / 12, dj, 2 / 12, -1)[0].conj())
    mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
    gate("phase rad", np.abs(np.angle(np.exp(1j * (aw - ra))))[mask], 1e-4)
    np.testing.assert_allclose(coi, rcoi, rtol=1e-12)


def _filter_cases(pywt_filters, seed=31, count=12):
    rng = np.random.default_rng(seed)
    names = sorted(k for k, v in pywt_filters.items() if len(v["dec_lo"]) <= 20)
    out = []
    for i in range(count * SCALE):
        n = int(np.exp(rng.uniform(np.log(16), np.log(40000))))
        name = str(rng.choice(names))
        out.append((i, n, name))
    return out


@pytest.fixture(scope="module")
def filters():
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "pywt_filters.json")) as f:
        return json.load(f)["filters"]


def _filter_ids():
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "pywt_filters.json")) as f:
        return _filter_cases(json.load(f)["filters"])


@pytest.mark.parametrize("case", _filter_ids(), ids=lambda c: f"bank{c[0]}-{c[2]}-n{c[1]}")
def test_random_modwt_and_dwt_match_oracle(case, filters):
    from wtmi import ops
    i, n, name = case
    fb = {k: np.asarray(v) for k, v in filters[name].items()}
    rng = np.random.default_rng(3000 + i)
    B = int(rng.integers(1, 4))
    x = np.stack([red_series(rng, n) for _ in range(B)])
    xd = torch.tensor(x, device="cuda")
    # MODWT: J up to the level where the dilated filter still fits 4 times
    J = int(rng.integers(1, max(2, min(12, int(np.log2(n)) - 1))))
    C = ops.modwt(xd, fb["dec_lo"], fb["dec_hi"], J).cpu().numpy()
    back = ops.imodwt(torch.tensor(C, device="cuda"), fb["dec_lo"], fb["dec_hi"]).cpu().numpy()
    for b in range(B):
        ref = ms.modwt_direct(x[b].astype(np.float64), fb["dec_lo"], fb["dec_hi"], J)
        gate(f"modwt[{b}] J={J}", row_relerr(C[b].astype(np.float64), ref))
        gate(f"round trip[{b}]", np.abs(back[b] - x[b]).max() / np.abs(x[b]).max())
    # DWT: pywt's maximum level for the length, or fewer
    lmax = ds.dwt_max_level(n, len(fb["dec_lo"]))
    if lmax < 1:
        return
    level = int(rng.integers(1, lmax + 1))
    coeffs, lens = ops.wavedec(xd, fb["dec_lo"], fb["dec_hi"], level)
    got = coeffs.cpu().numpy()
    for b in range(B):
        ref = np.concatenate(ds.wavedec(x[b].astype(np.float64), fb["dec_lo"], fb["dec_hi"], level))
        assert got[b].shape == ref.shape
        gate(f"wavedec[{b}] L={level}", np.abs(got[b] - ref).max() / np.abs(ref).max())
    rec = ops.waverec(coeffs, n, fb["rec_lo"], fb["rec_hi"], level, [(1 << (level + 1)) - 1]).cpu().numpy()
    for b in range(B):
        gate(f"waverec[{b}]", np.abs(rec[b, 0, :n] - x[b]).max() / np.abs(x[b]).max())


def _xwt_cases(seed=404, count=10):
    rng = np.random.default_rng(seed)
    mothers = [None, pc.Paul(4), pc.DOG(2), pc.MexicanHat(), pc.DOG(3), pc.Paul(6)]
    out = []
    for i in range(count * SCALE):
        n0 = int(np.exp(rng.uniform(np.log(12), np.log(16384))))
        dj = float(rng.choice([1 / 4, 1 / 8, 1 / 12]))
        m = mothers[i % len(mothers)]
        out.append((i, n0, dj, m))
    return out


def _mname(m):
    return "morlet" if m is None else f"{m.name}{getattr(m, 'm', '')}"


@pytest.mark.parametrize("case", _xwt_cases(), ids=lambda c: f"xwt{c[0]}-{_mname(c[3])}-n{c[1]}")
def test_random_xwt_pair_and_mothers_match_oracle(case):
    """The XWT pair kernel (W12, |W12|^2, significance ratio) and the non-Morlet mothers of the
    reference's MOTHER_DICT (Paul, DOG, Mexican hat; VAR = 1 kernels) at random shapes."""
    from wtmi import ops
    i, n0, dj, mother = case
    rng = np.random.default_rng(4000 + i)
    B = 2
    y1 = np.stack([red_series(rng, n0) for _ in range(B)])
    y2 = (0.6 * np.roll(y1, 3, axis=1) + 0.8 * np.stack([red_series(rng, n0) for _ in range(B)])
          ).astype(np.float32)
    dt, s0 = 1 / 12, 2 / 12
    wl = mother or pc.Morlet(6)
    J = max(1, min(int(np.round(np.log2(n0 * dt / s0) / dj)), 120))
    sj = s0 * 2 ** (np.arange(J + 1) * dj)
    ss = np.linspace(0.5, 2.0, sj.size)
    r = ops.xwt_morlet(torch.tensor(y1, device="cuda"), torch.tensor(y2, device="cuda"), sj, dt,
                       sig_scale=ss, want_w12=True, want_power=True, want_sig=True,
                       mother=mother)
    for b in range(B):
        W1 = pc.cwt(y1[b].astype(np.float64), dt, dj, s0, J, wl)[0]
        W2 = pc.cwt(y2[b].astype(np.float64), dt, dj, s0, J, wl)[0]
        W12 = W1 * W2.conj()
        # rows where the reference carries energy (Paul rows of a short series at the largest
        # scales can vanish to the fp64 floor, as in test_gpu_mothers)
        nrm = np.linalg.norm(W12, axis=-1)
        keep = nrm > 1e-6 * nrm.max()
        g = r["w12"][b].cpu().numpy().astype(np.complex128)
        gate(f"W12[{b}]", row_relerr(g[keep], W12[keep]))
        p = r["power"][b].cpu().numpy().astype(np.float64)
        gate(f"xwt power[{b}]", row_relerr(p[keep], (np.abs(W12) ** 2)[keep]))
        sg = r["sig"][b].cpu().numpy().astype(np.float64)
        gate(f"xwt sig ratio[{b}]", row_relerr(sg[keep], (np.abs(W12) ** 2 * ss[:, None])[keep]))


@pytest.mark.parametrize("case", _filter_ids()[:8 * SCALE], ids=lambda c: f"mra{c[0]}-{c[2]}-n{c[1]}")
def test_random_modwt_masks_match_oracle(case, filters):
    """MODWT multiresolution pieces (imodwt with a row keep-mask, the engine's MRA / smoothing
    path) at random lengths and filter banks against the oracle's masked synthesis."""
    from wtmi import ops
    i, n, name = case
    fb = {k: np.asarray(v) for k, v in filters[name].items()}
    rng = np.random.default_rng(5000 + i)
    x = red_series(rng, n)[None, :]
    J = int(rng.integers(1, max(2, min(10, int(np.log2(n)) - 1))))
    C = ops.modwt(torch.tensor(x, device="cuda"), fb["dec_lo"], fb["dec_hi"], J)
    Ch = C.cpu().numpy().astype(np.float64)[0]
    for keep in (1 << J, 1, (1 << (J + 1)) - 2, int(rng.integers(1, 1 << (J + 1)))):
        got = ops.imodwt(C, fb["dec_lo"], fb["dec_hi"], keep).cpu().numpy()[0]
        wm = Ch * np.array([(keep >> r) & 1 for r in range(J + 1)])[:, None]
        ref = ms.imodwt_direct(wm, fb["dec_lo"], fb["dec_hi"])
        gate(f"masked imodwt keep={keep:#x}", np.abs(got - ref).max() / max(np.abs(Ch).max(), 1e-30), 3e-5)
