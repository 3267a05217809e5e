"""CWT / XWT kernel parity vs the fp64 oracle (pycwt restatement).

Tolerance: per (series, scale) row ||W - W_ref|| / ||W_ref|| <= 1e-5.
Parity is against the restated pycwt algorithm (pycwt itself is absent: "parity
unpinned", pinned by tests/test_oracle_cwt.py known answers).
"""

import numpy as np
import pytest
import torch

from gpu_helpers import gate, red_series, row_relerr
from oracle import pycwt_spec as pc

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _ops():
    from wtmi import ops
    return ops


def _scales(n0, dt, dj, s0, J):
    return s0 * 2 ** (np.arange(J + 1) * dj)


@pytest.mark.parametrize("n0,dj,J", [(5, 1 / 4, 6), (8, 1 / 4, 8), (16, 1 / 4, 12),
                                     (37, 1 / 8, 30), (100, 1 / 8, 40), (256, 1 / 8, 50),
                                     (1000, 1 / 12, 70), (1333, 1 / 12, 84), (2048, 1 / 12, 90),
                                     (4096, 1 / 12, 127), (8192, 1 / 8, 96), (16384, 1 / 4, 50)])
def test_cwt_rows_match_oracle(n0, dj, J):
    rng = np.random.default_rng(n0)
    B = 3
    x = np.stack([red_series(rng, n0) for _ in range(B)])
    dt, s0 = 1 / 12, 2 / 12
    sj = _scales(n0, dt, dj, s0, J)
    xd = torch.tensor(x, device="cuda")
    ss = 1.0 / (1.0 + np.arange(sj.size))
    r = _ops().cwt_morlet(xd, sj, dt, 6.0, sig_scale=ss, want_w=True, want_power=True,
                          want_sig=True)
    torch.cuda.synchronize()
    W = r["w"].cpu().numpy()
    P = r["power"].cpu().numpy()
    Sg = r["sig"].cpu().numpy()
    assert W.shape == (B, sj.size, n0) and W.dtype == np.complex64
    for b in range(B):
        ref = pc.cwt(x[b].astype(np.float64), dt, dj, s0, J)[0]
        gate(f"W[{b}]", row_relerr(W[b].astype(np.complex128), ref), TOL)
        gate(f"power[{b}]", row_relerr(P[b].astype(np.float64), np.abs(ref) ** 2), TOL)
    np.testing.assert_allclose(Sg, P * ss[None, :, None], rtol=1e-6)


@pytest.mark.parametrize("n0,dj,J,offset", [(4096, 1 / 12, 127, 0.0), (4096, 1 / 12, 127, 500.0),
                                            (8192, 1 / 24, 255, 0.0), (2000, 1 / 12, 110, 50.0)])
def test_band_pruned_rows(n0, dj, J, offset):
    """Rows whose filtered spectrum lies in bins [0, N/16^q) enter the inverse FFT at pass q
    (cwt_common.hpp band_regime); full-band rows run a first pass over their NZ non-zero
    inputs only (first_pass_nz).  Random walks with a large mean put most of the energy at
    the lowest bins -- the worst case for the dropped negative-frequency tail."""
    rng = np.random.default_rng(n0 + 7)
    B = 2
    x = np.stack([red_series(rng, n0) for _ in range(B)]).astype(np.float64)
    x[1] = np.cumsum(rng.standard_normal(n0)) + offset
    x = x.astype(np.float32)
    dt, s0 = 1 / 12, 2 / 12
    sj = _scales(n0, dt, dj, s0, J)
    xd = torch.tensor(x, device="cuda")
    from wtmi import _lib
    with _lib.option("cwt_prune", 0):
        full = _ops().cwt_morlet(xd, sj, dt)["w"].cpu().numpy()
    for mode in (1, 2):  # band-pruned rows; + narrowed first passes of full-band rows
        with _lib.option("cwt_prune", mode):
            pr = _ops().cwt_morlet(xd, sj, dt)["w"].cpu().numpy()
        gate(f"pruned{mode} vs full", row_relerr(pr.astype(np.complex128), full.astype(np.complex128)), TOL)
        for b in range(B):
            ref = pc.cwt(x[b].astype(np.float64), dt, dj, s0, J)[0]
            gate(f"pruned{mode} W[{b}]", row_relerr(pr[b].astype(np.complex128), ref), TOL)


def test_many_scales_span_several_chunks():
    rng = np.random.default_rng(99)
    n0, dt, dj, s0, J = 300, 1 / 12, 1 / 64, 2 / 12, 600  # S = 601 > 512-row chunk table
    x = red_series(rng, n0)
    sj = _scales(n0, dt, dj, s0, J)
    W = _ops().cwt_morlet(torch.tensor(x, device="cuda"), sj, dt)["w"][0].cpu().numpy()
    ref = pc.cwt(x.astype(np.float64), dt, dj, s0, J)[0]
    assert row_relerr(W.astype(np.complex128), ref).max() < TOL


def test_affine_preprocessing_fused_in_load():
    rng = np.random.default_rng(5)
    n0, dt = 700, 1 / 12
    x = (red_series(rng, n0) + 40.0 + 0.05 * np.arange(n0)).astype(np.float32)
    a0, a1, a2 = 39.0, 0.05, 1 / 3.0
    sj = _scales(n0, dt, 1 / 12, 2 * dt, 60)
    aff = torch.tensor([[a0, a1, a2]], dtype=torch.float64, device="cuda")
    W = _ops().cwt_morlet(torch.tensor(x, device="cuda"), sj, dt, affine=aff)["w"][0].cpu().numpy()
    xs = ((x.astype(np.float64) - a0 - a1 * np.arange(n0)) * a2).astype(np.float32)
    ref = pc.cwt(xs.astype(np.float64), dt, 1 / 12, 2 * dt, 60)[0]
    assert row_relerr(W.astype(np.complex128), ref).max() < TOL


@pytest.mark.parametrize("n0", [64, 1333, 4096])
def test_xwt_pair_outputs(n0):
    rng = np.random.default_rng(n0 + 1)
    B = 2
    y1 = np.stack([red_series(rng, n0) for _ in range(B)])
    y2 = (0.6 * np.roll(y1, 3, axis=1) + 0.8 * np.stack([red_series(rng, n0) for _ in range(B)])
          ).astype(np.float32)
    dt, dj, s0 = 1 / 12, 1 / 8, 2 / 12
    J = int(np.round(np.log2(n0 * dt / s0) / dj))
    sj = _scales(n0, dt, dj, s0, J)
    ss = np.linspace(0.5, 2.0, sj.size)
    r = _ops().xwt_morlet(torch.tensor(y1, device="cuda"), torch.tensor(y2, device="cuda"), sj, dt,
                          sig_scale=ss, want_w12=True, want_power=True, want_sig=True,
                          want_uv=True)
    torch.cuda.synchronize()
    for b in range(B):
        W1 = pc.cwt(y1[b].astype(np.float64), dt, dj, s0, J)[0]
        W2 = pc.cwt(y2[b].astype(np.float64), dt, dj, s0, J)[0]
        W12 = W1 * W2.conj()
        g = r["w12"][b].cpu().numpy().astype(np.complex128)
        gate(f"W12[{b}]", row_relerr(g, W12), TOL)
        p = r["power"][b].cpu().numpy().astype(np.float64)
        gate(f"xwt power[{b}]", row_relerr(p, np.abs(W12) ** 2), TOL)
        sg = r["sig"][b].cpu().numpy().astype(np.float64)
        gate(f"xwt sig ratio[{b}]", row_relerr(sg, np.abs(W12) ** 2 * ss[:, None]), TOL)
        ang = np.angle(W12)
        u, v = r["u"][b].cpu().numpy(), r["v"][b].cpu().numpy()
        mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
        np.testing.assert_allclose(u[mask], np.cos(0.5 * np.pi - ang)[mask], atol=1e-4)
        np.testing.assert_allclose(v[mask], np.sin(0.5 * np.pi - ang)[mask], atol=1e-4)


def test_rejects_cpu_tensors_and_bad_args():
    ops = _ops()
    with pytest.raises(RuntimeError):
        ops.cwt_morlet(torch.zeros(1, 16), [1.0], 1.0)
    from wtmi import _lib
    with pytest.raises(_lib.WtmiError):
        _lib.call("wtmi_cwt_morlet", None, 0, 1, 16, None, None, 1, 1.0, 6.0, None, 0, None, None,
                  None, None, None)


def test_torch_custom_ops_match_oracle(db4):
    import wtmi.ops  # noqa: F401  (registers torch.ops.wtmi)
    from oracle import modwt_spec as ms
    rng = np.random.default_rng(21)
    n0, dt = 512, 1 / 12
    x = np.stack([red_series(rng, n0) for _ in range(2)])
    sj = _scales(n0, dt, 1 / 8, 2 * dt, 40)
    xd = torch.tensor(x, device="cuda")
    W = torch.ops.wtmi.cwt(xd, torch.tensor(sj, device="cuda"), dt, 6.0).cpu().numpy()
    ref = pc.cwt(x[1].astype(np.float64), dt, 1 / 8, 2 * dt, 40)[0]
    assert row_relerr(W[1].astype(np.complex128), ref).max() < TOL
    lo = torch.tensor(db4["dec_lo"])
    hi = torch.tensor(db4["dec_hi"])
    w = torch.ops.wtmi.modwt(xd, lo, hi, 4)
    r = ms.modwt(x[0].astype(np.float64), db4["dec_lo"], db4["dec_hi"], 4)
    assert np.abs(w[0].cpu().numpy() - r).max() <= 1e-5 * np.abs(r).max()
    xr = torch.ops.wtmi.imodwt(w, lo, hi).cpu().numpy()
    assert np.abs(xr - x).max() <= 1e-5 * np.abs(x).max()


def test_torch_custom_ops_xwt_dwt_stats(db4):
    """torch.ops.wtmi.{xwt, xwt_power, dwt, idwt, series_stats} vs the oracle, and their
    fake (meta) kernels agree with the real output shapes."""
    import wtmi.ops  # noqa: F401
    from oracle import dwt_spec as ds
    from torch._subclasses.fake_tensor import FakeTensorMode
    rng = np.random.default_rng(22)
    n0, dt, dj, J = 700, 1 / 12, 1 / 8, 50
    x1 = np.stack([red_series(rng, n0) for _ in range(2)])
    x2 = np.stack([red_series(rng, n0) for _ in range(2)])
    sj = torch.tensor(_scales(n0, dt, dj, 2 * dt, J), device="cuda")
    d1, d2 = torch.tensor(x1, device="cuda"), torch.tensor(x2, device="cuda")
    W12 = torch.ops.wtmi.xwt(d1, d2, sj, dt, 6.0)
    P = torch.ops.wtmi.xwt_power(d1, d2, sj, dt, 6.0)
    ref = (pc.cwt(x1[1].astype(np.float64), dt, dj, 2 * dt, J)[0]
           * pc.cwt(x2[1].astype(np.float64), dt, dj, 2 * dt, J)[0].conj())
    gate("op xwt W12", row_relerr(W12[1].cpu().numpy().astype(np.complex128), ref), TOL)
    gate("op xwt_power", row_relerr(P[1].cpu().numpy().astype(np.float64), np.abs(ref) ** 2), TOL)
    lo, hi = torch.tensor(db4["dec_lo"]), torch.tensor(db4["dec_hi"])
    rlo, rhi = torch.tensor(db4["rec_lo"]), torch.tensor(db4["rec_hi"])
    C = torch.ops.wtmi.dwt(d1, lo, hi, 5)
    flat = np.concatenate(ds.wavedec(x1[0].astype(np.float64), db4["dec_lo"], db4["dec_hi"], 5))
    assert C.shape[1] == flat.size and np.abs(C[0].cpu().numpy() - flat).max() <= 1e-5 * np.abs(flat).max()
    back = torch.ops.wtmi.idwt(C, n0, rlo, rhi, 5).cpu().numpy()
    assert back.shape == (2, n0) and np.abs(back - x1).max() <= 1e-5 * np.abs(x1).max()
    st = torch.ops.wtmi.series_stats(d1).cpu().numpy()
    np.testing.assert_allclose(st[:, 0], x1.astype(np.float64).mean(axis=1), rtol=1e-9)
    np.testing.assert_allclose(st[:, 1], x1.astype(np.float64).std(axis=1), rtol=1e-9)
    with FakeTensorMode(allow_non_fake_inputs=True):
        f1 = torch.empty(2, n0, device="cuda")
        fs = torch.empty(sj.numel(), dtype=torch.float64, device="cuda")
        assert torch.ops.wtmi.xwt(f1, f1, fs, dt, 6.0).shape == W12.shape
        assert torch.ops.wtmi.dwt(f1, lo, hi, 5).shape == C.shape
        assert torch.ops.wtmi.series_stats(f1).shape == (2, 8)
